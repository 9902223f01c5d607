#!/usr/bin/env python
"""Diagnostic: run attention fwd on fixed inputs (model shapes) and save outputs, so
two library builds can be compared bitwise.  python scripts/diag/attn_dump.py <out.pt>"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from multimodal_llm_pretraining_amd import kernels as K  # noqa: E402

torch.manual_seed(0)
res = {}
for (name, B, S, H, D, causal, hs, ps) in [("text", 2, 707, 8, 256, True, 768, 256),
                                           ("vit", 2, 197, 12, 64, False, 64, 768)]:
    T = B * S
    qkv = (torch.randn(T, 3 * H * D, device="cuda") * 1.5).to(torch.bfloat16)
    out = torch.empty(T, H * D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B * H * S, device="cuda")
    K.attention_fwd(qkv, B, S, H, D, hs, ps, causal, D ** -0.5, out, lse)
    res[name] = out.cpu()
    res[name + "_lse"] = lse.cpu()
torch.save(res, sys.argv[1])
if len(sys.argv) > 2:
    ref = torch.load(sys.argv[2])
    for k, v in res.items():
        d = (v.float() - ref[k].float()).abs()
        print(k, "bitwise-equal" if torch.equal(v, ref[k]) else f"differs: {(d > 0).sum().item()} elems, max {d.max().item():.3e}")
