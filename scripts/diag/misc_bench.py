"""Micro-benchmark of the weight transpose (W^T shadow refresh) and the partial-rotary kernel at
C5's shapes (Pythia-2.8B: hidden 2560, 32 heads of 80, rotary 20; CLIP-L/14-336 tower), one
JSON line per case with the achieved HBM rate."""
import json
import sys

import torch

sys.path.insert(0, ".")
from multimodal_llm_pretraining_amd import kernels as K  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e-3


def main():
    dev = "cuda"
    for rows, cols in [(7680, 2560), (2560, 2560), (10240, 2560), (2560, 10240), (3072, 1024),
                       (4096, 1024), (1024, 4096), (6144, 2048), (2048, 8192)]:
        src = torch.randn(rows, cols, device=dev).to(torch.bfloat16)
        dst = torch.empty(cols, rows, device=dev, dtype=torch.bfloat16)
        t = timeit(lambda: K.transpose_bf16(src, dst))
        assert torch.equal(dst, src.t())
        print(json.dumps({"kernel": "transpose", "rows": rows, "cols": cols, "us": round(t * 1e6, 1),
                          "GBps": round(2 * rows * cols * 2 / t / 1e9, 1)}), flush=True)
    T, seq, heads, hd, rot = 64 * 1087, 1087, 32, 80, 20
    qkv = torch.randn(T, 3 * heads * hd, device=dev).to(torch.bfloat16)
    pos = torch.arange(seq, dtype=torch.float32, device=dev)[:, None]
    inv = 1.0 / (10000 ** (torch.arange(0, rot, 2, device=dev).float() / rot))
    ang = torch.cat([pos * inv, pos * inv], 1)
    cos, sin = ang.cos().contiguous(), ang.sin().contiguous()
    t = timeit(lambda: K.rope_inplace(qkv, seq, heads, hd, rot, 3 * hd, hd, cos, sin))
    moved = T * heads * 2 * rot * 2 * 2  # q and k rotary dims, read + write
    print(json.dumps({"kernel": "rope", "tokens": T, "heads": heads, "head_dim": hd, "rot": rot,
                      "us": round(t * 1e6, 1), "GBps_rot_bytes": round(moved / t / 1e9, 1)}),
          flush=True)

    for rows, h in [(64 * 1087, 2560), (256 * 707, 2048), (64 * 577, 1024)]:
        x = torch.randn(rows, h, device=dev)
        mean, rstd = x.mean(1), torch.rsqrt(x.var(1, unbiased=False) + 1e-5)
        dy1 = torch.randn(rows, h, device=dev).to(torch.bfloat16)
        dy2 = torch.randn(rows, h, device=dev).to(torch.bfloat16)
        w1, w2 = torch.randn(h, device=dev), torch.randn(h, device=dev)
        dres = torch.randn(rows, h, device=dev)
        dx = torch.empty(rows, h, device=dev)
        dxb = torch.empty(rows, h, device=dev, dtype=torch.bfloat16)
        g = [torch.zeros(h, device=dev) for _ in range(6)]
        t = timeit(lambda: K.layernorm_bwd(x, mean, rstd, dy1, w1, dx, g[0], g[1], dy2, w2, g[2], g[3],
                                           dres, dxb, g[4], g[5]))
        moved = rows * h * (4 + 2 + 2 + 4 + 4 + 2)  # x, dy1, dy2, dresid in; dx, dx_bf16 out
        print(json.dumps({"kernel": "layernorm_bwd_ex", "rows": rows, "h": h, "us": round(t * 1e6, 1),
                          "GBps": round(moved / t / 1e9, 1)}), flush=True)
        del x, dy1, dy2, dres, dx, dxb
        torch.cuda.empty_cache()

    n = 1_103_942_144  # C3's parameters: one fused AdamW + bf16 shadow + zero_grad
    pf, g, m, v = (torch.randn(n, device=dev) for _ in range(4))
    pb = torch.empty(n, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: K.adam_step(pf, g, m, v, pb, lr=1e-4, beta1=0.9, beta2=0.999, eps=1e-8,
                                   weight_decay=0.0, adamw=True, step=3, zero_grad=True), 10)
    print(json.dumps({"kernel": "adam_zero_grad", "params": n, "us": round(t * 1e6, 1),
                      "GBps": round(34 * n / t / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
