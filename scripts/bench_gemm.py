#!/usr/bin/env python
"""GEMM microbenchmark on the exact shapes of the ViT-B/16+Pythia-1B step
(micro-batch 64 → T = 64·707 tokens): the libmmpt kernel per (layout, epilogue)
vs torch.matmul (hipBLASLt) on the same bf16 operands as a library yardstick.
Random operands (cdna_hip_programming.md rule 25).  Prints one JSON line per shape.

python scripts/bench_gemm.py [--tokens 45248] [--iters 20]
"""

from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from multimodal_llm_pretraining_amd import kernels as K  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=64 * 707)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--no-ref", action="store_true")
    ap.add_argument("--only", default="", help="comma-separated shape names")
    ap.add_argument("--vit-tokens", type=int, default=256 * 197)
    ap.add_argument("--bias", action="store_true", help="bias on the forward shapes (as the model)")
    ap.add_argument("--clip-tokens", type=int, default=64 * 577, help="CLIP-L/14-336 tower rows")
    args = ap.parse_args()
    T = args.tokens
    V = args.vit_tokens
    dev = "cuda"
    shapes = [  # (name, kind, rows-out, cols-out, contraction)
        ("qkv_fwd", "fwd", T, 6144, 2048), ("dense_fwd", "fwd", T, 2048, 2048),
        ("fc1_fwd_gelu", "fwd_gelu", T, 8192, 2048), ("fc1_fwd_plain", "fwd", T, 8192, 2048),
        ("fc2_fwd_resid", "fwd_resid", T, 2048, 8192), ("fc2_fwd_plain", "fwd", T, 2048, 8192),
        ("lm_head_fwd", "fwd", T, 50304, 2048),
        ("qkv_dx", "dx", T, 2048, 6144), ("fc1_dx", "dx", T, 2048, 8192),
        ("fc2_dx_dgelu", "dx_dgelu", T, 8192, 2048), ("fc2_dx_plain", "dx", T, 8192, 2048),
        ("lm_head_dx", "dx", T, 2048, 50304),
        ("qkv_dw", "dw", 6144, 2048, T), ("dense_dw", "dw", 2048, 2048, T),
        ("fc1_dw", "dw", 8192, 2048, T), ("fc2_dw", "dw", 2048, 8192, T), ("lm_head_dw", "dw", 50304, 2048, T),
        ("vit_fc1_fwd", "fwd_gelu", 64 * 197, 3072, 768), ("vit_fc1_dw", "dw", 3072, 768, 64 * 197),
        ("vit_qkv_fwd", "fwd", V, 2304, 768), ("vit_o_fwd", "fwd", V, 768, 768),
        ("vit_fc1_fwd_big", "fwd_gelu", V, 3072, 768), ("vit_fc2_fwd", "fwd_resid", V, 768, 3072),
        ("vit_qkv_dx", "dx", V, 768, 2304), ("vit_fc1_dx", "dx", V, 768, 3072),
        ("vit_fc2_dx", "dx_dgelu", V, 3072, 768), ("vit_qkv_dw", "dw", 2304, 768, V),
        ("vit_fc1_dw_big", "dw", 3072, 768, V),
        ("fc2_dx_dgelu_cs", "dgelu_cs", T, 8192, 2048),
        ("fc1_dw_bt", "dw_bt", 8192, 2048, T), ("fc1_dw_both", "dw_both", 8192, 2048, T),
        ("qkv_dw_bt", "dw_bt", 6144, 2048, T), ("qkv_dw_both", "dw_both", 6144, 2048, T),
        # the input-gradient GEMMs as the engine runs them: dY x the transposed weight shadow,
        # both operands K-contiguous (lm_head over the 511/707 scored rows)
        ("qkv_dxt", "dxt", T, 2048, 6144), ("dense_dxt", "dxt", T, 2048, 2048),
        ("fc1_dxt", "dxt", T, 2048, 8192), ("lm_head_dxt", "dxt", T * 511 // 707, 2048, 50304),
        ("lm_head_dw_sc", "dw", 50304, 2048, T * 511 // 707),
        # round 5: the quick-GELU (CLIP-L tower) and SwiGLU (Llama-3.2-1B) forms on gemm4p
        ("clip_fc1_qgelu", "fwd_qgelu", args.clip_tokens, 4096, 1024),
        ("clip_fc2_dx_dqgelu", "dxt_dqgelu", args.clip_tokens, 4096, 1024),
        ("llama_gate_up_swiglu", "fwd_swiglu", T, 16384, 2048),
        ("llama_down_dx_dswiglu", "dxt_dswiglu", T, 8192, 2048),
        # round 5: weight + bias gradient in one pass (EPI_F32_ACC_COLSUM + the partial reduce)
        ("qkv_dw_cs", "dw_cs", 6144, 2048, T), ("vit_qkv_dw_cs", "dw_cs", 2304, 768, V),
        # round 6: Pythia-2.8B's weight gradients (C5, T = 64 x 1087 = 69,568 tokens)
        ("p28_fc1_dw", "dw", 10240, 2560, T), ("p28_fc2_dw", "dw", 2560, 10240, T),
        ("p28_qkv_dw", "dw", 7680, 2560, T), ("p28_dense_dw", "dw", 2560, 2560, T),
        ("p28_qkv_dw_cs", "dw_cs", 7680, 2560, T),
        ("sq4096", "fwd", 4096, 4096, 4096), ("sq8192", "fwd", 8192, 8192, 8192),
        ("sq8192_dx", "dx", 8192, 8192, 8192), ("sq8192_dw", "dw", 8192, 8192, 8192),
    ]
    torch.manual_seed(0)
    only = set(args.only.split(",")) if args.only else None
    for name, kind, M, N, Kd in shapes:
        if only and name not in only:
            continue
        flops = 2.0 * M * N * Kd
        if kind == "dgelu_cs":  # the model's fc2 dX + dGELU + fc1 bias column sums (W^T shadow)
            a = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
            b = (torch.randn(N, Kd, device=dev) * 0.02).to(torch.bfloat16)
            pre_t = torch.randn(M, N, device=dev).to(torch.bfloat16)
            db = torch.zeros(N, device=dev)
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            t = timeit(lambda: K.gemm_dgelu_colsum(a, b, out, pre_t, db), args.iters)
            print(json.dumps({"shape": name, "M": M, "N": N, "K": Kd,
                              "mmpt_tflops": round(flops / t / 1e12, 1), "mmpt_us": round(t * 1e6, 1)}),
                  flush=True)
            del a, b, out, pre_t
            torch.cuda.empty_cache()
            continue
        if kind.startswith("fwd") or kind.startswith("dxt"):
            a = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
            b = (torch.randn(N, Kd, device=dev) * 0.02).to(torch.bfloat16)
            la, lb = K.ROWS_K, K.ROWS_K
            ref = lambda: a @ b.t()  # noqa: E731
        elif kind.startswith("dx"):
            a = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
            b = (torch.randn(Kd, N, device=dev) * 0.02).to(torch.bfloat16)
            la, lb = K.ROWS_K, K.K_ROWS
            ref = lambda: a @ b  # noqa: E731
        elif kind == "dw_bt":  # weight gradient with B pre-transposed (K-contiguous)
            a = torch.randn(Kd, M, device=dev).to(torch.bfloat16)
            b = torch.randn(N, Kd, device=dev).to(torch.bfloat16)
            la, lb = K.K_ROWS, K.ROWS_K
            ref = lambda: a.t() @ b.t()  # noqa: E731
        elif kind == "dw_both":  # both operands K-contiguous (layout yardstick)
            a = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
            b = torch.randn(N, Kd, device=dev).to(torch.bfloat16)
            la, lb = K.ROWS_K, K.ROWS_K
            ref = lambda: a @ b.t()  # noqa: E731
        else:
            a = torch.randn(Kd, M, device=dev).to(torch.bfloat16)
            b = torch.randn(Kd, N, device=dev).to(torch.bfloat16)
            la, lb = K.K_ROWS, K.K_ROWS
            ref = lambda: a.t() @ b  # noqa: E731
        kw = {}
        if args.bias and kind.startswith("fwd") and kind != "fwd_swiglu":
            kw["bias"] = (torch.randn(N, device=dev) * 0.1).to(torch.bfloat16)
        if kind.startswith("dw"):
            out = torch.zeros(M, N, device=dev)
            kw["epilogue"] = K.EPI_F32_ACC
        elif kind == "fwd_resid":
            out = torch.empty(M, N, device=dev)
            kw.update(epilogue=K.EPI_F32_RESID, out2=torch.randn(M, N, device=dev),
                      aux=torch.randn(M, N, device=dev).to(torch.bfloat16))
        elif kind == "dxt_dswiglu":  # d act GEMM -> (d gate, d up), blocked [M][2N]
            out = torch.empty(M, 2 * N, device=dev, dtype=torch.bfloat16)
            kw.update(epilogue=K.EPI_BF16_DSWIGLU,
                      aux=torch.randn(M, 2 * N, device=dev).to(torch.bfloat16))
        else:
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            if kind == "fwd_qgelu":
                kw.update(epilogue=K.EPI_BF16_QGELU, out2=torch.empty_like(out))
            elif kind == "fwd_swiglu":
                kw.update(epilogue=K.EPI_BF16_SWIGLU,
                          out2=torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16))
            elif kind == "dxt_dqgelu":
                kw.update(epilogue=K.EPI_BF16_DQGELU, aux=torch.randn(M, N, device=dev).to(torch.bfloat16))
            elif kind == "fwd_gelu":
                kw.update(epilogue=K.EPI_BF16_GELU, out2=torch.empty_like(out))
            elif kind == "dx_dgelu":
                kw.update(epilogue=K.EPI_BF16_DGELU, aux=torch.randn(M, N, device=dev).to(torch.bfloat16))
        if kind == "dw_cs":
            db = torch.zeros(M, device=dev)
            if not K.gemm_wgrad_colsum(a, b, out, db):  # fused form not taken: nothing to time
                print(json.dumps({"shape": name, "M": M, "N": N, "K": Kd, "fused": False}), flush=True)
                continue
            t = timeit(lambda: K.gemm_wgrad_colsum(a, b, out, db), args.iters)
        else:
            t = timeit(lambda: K.gemm(a, b, out, layout_a=la, layout_b=lb, **kw), args.iters)
        rec = {"shape": name, "M": M, "N": N, "K": Kd, "mmpt_tflops": round(flops / t / 1e12, 1),
               "mmpt_us": round(t * 1e6, 1), "kernel": K.gemm_last_kernel()}
        if not args.no_ref:
            tr = timeit(ref, args.iters)
            rec["hipblaslt_tflops"] = round(flops / tr / 1e12, 1)
        print(json.dumps(rec), flush=True)
        del a, b, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
