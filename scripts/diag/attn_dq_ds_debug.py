"""Diagnostic: D = 256 attention backward with and without dS tiles (MMPT_ATTN_DS) on one
small causal shape; reports where dQ / dK / dV differ or are non-finite.  Runs each mode in
a child process (the switch is read once per process)."""
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def run(out):
    from multimodal_llm_pretraining_amd import kernels as K
    B, S, H, D = 2, 641, 2, 256
    g = torch.Generator(device="cuda").manual_seed(3)
    qkv = torch.randn(B * S, 3 * H * D, device="cuda", generator=g).to(torch.bfloat16)
    dout = torch.randn(B * S, H * D, device="cuda", generator=g).to(torch.bfloat16)
    o = torch.empty(B * S, H * D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B * H * S, device="cuda")
    K.attention_fwd(qkv, B, S, H, D, 3 * D, D, True, D ** -0.5, o, lse)
    dq = torch.zeros_like(qkv)
    K.attention_bwd(qkv, B, S, H, D, 3 * D, D, True, D ** -0.5, o, dout, lse, dq)
    torch.cuda.synchronize()
    torch.save(dq.cpu(), out)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run(sys.argv[1])
        sys.exit(0)
    res = {}
    for m in ("0", "1"):
        path = f"/tmp/dq_{m}.pt"
        subprocess.run([sys.executable, __file__, path], check=True, env={**os.environ, "MMPT_ATTN_DS": m})
        res[m] = torch.load(path).float().view(2, 641, 2, 3, 256)
    a, b = res["0"], res["1"]
    for part, name in ((0, "dq"), (1, "dk"), (2, "dv")):
        x, y = a[:, :, :, part], b[:, :, :, part]
        bad = ~torch.isfinite(y)
        diff = (x - y).abs()
        print(name, "nonfinite", int(bad.sum()), "maxdiff", float(diff[~bad].max()) if (~bad).any() else None,
              "ref max", float(x.abs().max()))
        if bad.any():
            rows = torch.nonzero(bad.any(-1))
            print("  nonfinite (b, s, h):", rows[:10].tolist(), "... rows", sorted(set(rows[:, 1].tolist()))[:40])
        rel = diff.amax(-1) / (x.abs().amax(-1) + 1e-6)
        worst = torch.nonzero(rel > 0.05)
        print("  rows rel > 5%:", worst.shape[0], sorted(set(worst[:, 1].tolist()))[:40])
