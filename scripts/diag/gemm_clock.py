"""Diagnostic (GPU, the MMPT_GEMM_DIAG=7 library: MMPT_LIB=.../libmmpt_clock.so): the in-kernel
clock of the big-tile GEMM kernels (MI355X_MICROARCH.md 'DVFS give-back' item 6) — per
workgroup Δs_memtime / Δs_memrealtime × 100 MHz, median over the workgroups of the last launch
after >= 2 s of back-to-back launches on random data — beside the launch's wall time and
TF/s.  Run it once per arm on the same box (round 5 compared MMPT_GEMM_4P=1: gemm4p against =0:
the 8-wave gemm256 kernel, since retired)."""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from multimodal_llm_pretraining_amd import _lib  # noqa: E402
from multimodal_llm_pretraining_amd import kernels as K  # noqa: E402

SHAPES = {  # name: (M, N, K, layout) — C3's dominant forms at T = 180,992 plus the yardstick
    "sq8192": (8192, 8192, 8192, "fwd"),
    "qkv_fwd": (180992, 6144, 2048, "fwd"),
    "dense_dxt": (180992, 2048, 2048, "fwd"),
    "fc1_dw": (8192, 2048, 180992, "dw"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    ap.add_argument("--seconds", type=float, default=2.5)
    args = ap.parse_args()
    lib = _lib.load()
    fn = lib.mmpt_gemm_diag_clock  # AttributeError: not the diagnostic-7 library
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    fn.restype = ctypes.c_int
    dev = "cuda"
    torch.manual_seed(0)
    for name, (M, N, Kd, kind) in SHAPES.items():
        if args.only and name not in args.only.split(","):
            continue
        if kind == "fwd":
            a = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
            b = (torch.randn(N, Kd, device=dev) * 0.02).to(torch.bfloat16)
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            run = lambda: K.gemm(a, b, out)  # noqa: E731
        else:
            a = torch.randn(Kd, M, device=dev).to(torch.bfloat16)
            b = torch.randn(Kd, N, device=dev).to(torch.bfloat16)
            out = torch.zeros(M, N, device=dev)
            run = lambda: K.gemm(a, b, out, layout_a=K.K_ROWS, layout_b=K.K_ROWS,  # noqa: E731
                                 epilogue=K.EPI_F32_ACC)
        run()
        torch.cuda.synchronize()
        t0 = time.time()
        n = 0
        while time.time() - t0 < args.seconds:
            run()
            n += 1
            if n % 8 == 0:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run()
        e1.record()
        torch.cuda.synchronize()
        wall = e0.elapsed_time(e1) * 1e-3
        kname = K.gemm_last_kernel()
        nwg = 256
        buf = (ctypes.c_ulonglong * (4 * nwg))()
        rc = fn(buf, nwg)
        assert rc == 0, rc
        clocks, spans = [], []
        for w in range(nwg):
            c0, c1, r0, r1 = buf[4 * w: 4 * w + 4]
            if r1 > r0 and c1 > c0:
                clocks.append((c1 - c0) / (r1 - r0) * 100.0)  # MHz
                spans.append((r1 - r0) / 100.0)  # us
        rec = {"shape": name, "kernel": kname, "arm": os.environ.get("MMPT_GEMM_4P", "1"),
               "wall_us": round(wall * 1e6, 1), "tflops": round(2.0 * M * N * Kd / wall / 1e12, 1),
               "clock_mhz_median": round(statistics.median(clocks), 1) if clocks else None,
               "clock_mhz_min": round(min(clocks), 1) if clocks else None,
               "clock_mhz_max": round(max(clocks), 1) if clocks else None,
               "wg_span_us_median": round(statistics.median(spans), 1) if spans else None,
               "warm_launches": n}
        print(json.dumps(rec), flush=True)
        del a, b, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
