#!/usr/bin/env python
"""Attention forward accuracy vs an fp64 reference on the Pythia shape (diagnostic):
mean |err|, mean signed err and the bf16-rounding of the reference as a yardstick."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from multimodal_llm_pretraining_amd import kernels as K  # noqa: E402

torch.manual_seed(0)
for (B, S, H, D, causal, hs_mode) in [(2, 707, 8, 256, True, "il"), (4, 197, 12, 64, False, "pl")]:
    T = B * S
    qkv = (torch.randn(T, 3 * H * D, device="cuda") * 1.5).to(torch.bfloat16)
    hs, ps = (3 * D, D) if hs_mode == "il" else (D, H * D)
    out = torch.empty(T, H * D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B * H * S, device="cuda")
    K.attention_fwd(qkv, B, S, H, D, hs, ps, causal, D ** -0.5, out, lse)
    v = qkv.double().view(T, -1)
    def part(p):
        idx = torch.stack([torch.arange(D, device="cuda") + h * hs + p * ps for h in range(H)])
        return v[:, idx].view(B, S, H, D).transpose(1, 2)
    q, k, vv = part(0), part(1), part(2)
    sc = (q @ k.transpose(-1, -2)) * D ** -0.5
    if causal:
        sc = sc.masked_fill(~torch.ones(S, S, device="cuda", dtype=torch.bool).tril(), float("-inf"))
    ref = torch.softmax(sc, -1) @ vv
    got = out.view(B, S, H, D).transpose(1, 2).double()
    e = got - ref
    eb = ref.to(torch.bfloat16).double() - ref
    print(f"D={D}: mean|err| {e.abs().mean().item():.3e} mean err {e.mean().item():+.3e} "
          f"max {e.abs().max().item():.3e} | bf16(ref) mean|err| {eb.abs().mean().item():.3e}")
