#!/usr/bin/env python
"""Attention microbenchmark on the step's shapes: GPTNeoX (Pythia-1B: B=64, S=707, H=8,
D=256, causal, interleaved qkv), ViT-B/16 (B=64, S=197, H=12, D=64, planar qkv) and
Pythia-2.8B's head shape (B=16, S=707, H=32, D=80: the D = 128 kernels computing 80 dims,
MMPT_ATTN_NATIVE80=1, beside the zero-filled 128-dim path, =0).
Random N(0,1) activations (cdna_hip_programming.md rule 25).  Reports causal-exact
TFLOP/s (fwd 4·B·H·S²·D / 2, bwd 2.5× that) and the full-square convention.

python scripts/bench_attn.py [--iters 20]
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
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--long", action="store_true", help="add S = 2048 / 4096 causal D = 256 cases")
    args = ap.parse_args()
    torch.manual_seed(0)
    cases = [("pythia", 64, 707, 8, 256, True, "interleaved"), ("vit", 64, 197, 12, 64, False, "planar"),
             ("pythia_bench", 256, 707, 8, 256, True, "interleaved"),  # the headline micro-batch
             ("pythia28_native80", 16, 707, 32, 80, True, "interleaved"),
             ("pythia28_padded128", 16, 707, 32, 80, True, "interleaved"),
             ("pythia28_c5", 64, 1087, 32, 80, True, "interleaved")]  # C5's micro-batch 64 x 1087
    if args.long:
        cases += [("s2048", 22, 2048, 8, 256, True, "interleaved"),
                  ("s4096", 11, 4096, 8, 256, True, "interleaved")]
    from multimodal_llm_pretraining_amd import _lib

    for name, B, S, H, D, causal, layout in cases:
        if D == 80:
            _lib.set_switch("MMPT_ATTN_NATIVE80", 0 if name.endswith("padded128") else 1)
        T = B * S
        qkv = torch.randn(T, 3 * H * D, device="cuda").to(torch.bfloat16)
        if layout == "interleaved":
            hs, ps = 3 * D, D
        else:
            hs, ps = D, H * D
        out = torch.empty(T, H * D, device="cuda", dtype=torch.bfloat16)
        lse = torch.empty(B * H * S, device="cuda")
        dout = torch.randn(T, H * D, device="cuda").to(torch.bfloat16)
        dqkv = torch.empty_like(qkv)
        scale = D ** -0.5
        fwd = lambda: K.attention_fwd(qkv, B, S, H, D, hs, ps, causal, scale, out, lse)  # noqa: E731
        bwd = lambda: K.attention_bwd(qkv, B, S, H, D, hs, ps, causal, scale, out, dout, lse, dqkv)  # noqa: E731
        tf = timeit(fwd, args.iters)
        tb = timeit(bwd, args.iters)
        extra = {}
        if name == "pythia_bench":  # + the rope backward: fused (dK / dQ epilogues) vs a second pass
            from multimodal_llm_pretraining_amd.engine import rope_tables

            cos, sin = (t.cuda() for t in rope_tables(H * D, H, 0.25, 10000.0, S))
            rot = cos.shape[1]

            def two_pass():
                bwd()
                K.rope_inplace(dqkv, S, H, D, rot, hs, ps, cos, sin, inverse=True)

            fused = lambda: K.attention_bwd_rope(qkv, B, S, H, D, hs, ps, causal, scale, out, dout,  # noqa: E731
                                                 lse, dqkv, rot, cos, sin)
            extra = {"bwd_rope_two_pass_us": round(timeit(two_pass, args.iters) * 1e6, 1),
                     "bwd_rope_fused_us": round(timeit(fused, args.iters) * 1e6, 1)}
        full = 4.0 * B * H * S * S * D
        exact = full / 2 if causal else full
        print(json.dumps({"case": name, "ds_mode": os.environ.get("MMPT_ATTN_DS", "1"), "fwd_us": round(tf * 1e6, 1), "bwd_us": round(tb * 1e6, 1),
                          "fwd_tflops_exact": round(exact / tf / 1e12, 1),
                          "bwd_tflops_exact": round(2.5 * exact / tb / 1e12, 1),
                          "fwd_tflops_fullsq": round(full / tf / 1e12, 1), **extra}), flush=True)


if __name__ == "__main__":
    main()
