"""LayerNorm backward / forward at the step's Pythia shape (rows = 256 x 707, h = 2048, two LNs
on one input as GPT-NeoX's parallel residual): µs per call, one JSON line per kernel.
Diagnostic A/B only (MMPT_LIB selects a variant library)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from multimodal_llm_pretraining_amd import kernels as K  # noqa: E402

dev = "cuda"
rows, h = 256 * 707, 2048
torch.manual_seed(0)
x = torch.randn(rows, h, device=dev)
w1, b1 = torch.randn(h, device=dev), torch.randn(h, device=dev)
w2, b2 = torch.randn(h, device=dev), torch.randn(h, device=dev)
y1 = torch.empty(rows, h, device=dev, dtype=torch.bfloat16)
y2 = torch.empty_like(y1)
mean, rstd = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
dy1 = torch.randn(rows, h, device=dev).to(torch.bfloat16)
dy2 = torch.randn(rows, h, device=dev).to(torch.bfloat16)
dres = torch.randn(rows, h, device=dev)
dx = torch.empty(rows, h, device=dev)
dxb = torch.empty(rows, h, device=dev, dtype=torch.bfloat16)
g = [torch.zeros(h, device=dev) for _ in range(6)]


def fwd():
    K.layernorm_fwd(x, w1, b1, 1e-5, y1, mean, rstd, w2, b2, y2)


def bwd():
    K.layernorm_bwd(x, mean, rstd, dy1, w1, dx, g[0], g[1], dy2, w2, g[2], g[3], dresid=dres,
                    dx_bf16=dxb, dsum=g[4], dsum2=g[5])


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


fwd()
ref = None
for name, fn, gb in (("ln_fwd", fwd, rows * h * (4 + 2 + 2) / 1e9),
                     ("ln_bwd", bwd, rows * h * (4 + 2 + 2 + 4 + 4 + 2) / 1e9)):
    us = timeit(fn)
    print(json.dumps({"kernel": name, "us": round(us, 1), "GB": round(gb, 2),
                      "TBps": round(gb / us * 1e3, 2)}), flush=True)
bwd()
torch.cuda.synchronize()
print(json.dumps({"check": float(dx.double().abs().sum()), "dsum": float(g[4].double().abs().sum())}))
