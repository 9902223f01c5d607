"""Diagnostic: the dQGELU epilogue vs (a) torch bf16 autograd on the GPU, (b) the CPU,
(c) an explicit rounding emulation."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from multimodal_llm_pretraining_amd import kernels as K  # noqa: E402

torch.manual_seed(5)
M, N, Kd = 333, 264, 320
A = torch.randn(M, Kd, device="cuda").bfloat16()
W = (torch.randn(N, Kd, device="cuda") * 0.1).bfloat16()
pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
K.gemm(A, W, pre)
g = torch.empty_like(pre)
K.gemm(A, W, g)
dg = torch.empty_like(pre)
K.gemm(A, W, dg, epilogue=K.EPI_BF16_DQGELU, aux=pre)


def autograd(x, g):
    xr = x.clone().requires_grad_()
    (xr * torch.sigmoid(1.702 * xr)).backward(g)
    return xr.grad.float()


def emul(x, g):
    rb = lambda t: t.to(torch.bfloat16).float()  # noqa: E731
    xf, gf = x.float(), g.float()
    s = rb(torch.sigmoid(rb(1.702 * xf)))
    a = rb(gf * s)
    gt = rb(rb(gf * xf) * (1 - s) * s)
    return rb(a + rb(gt * 1.702))


for name, ref in (("gpu autograd", autograd(pre, g)), ("cpu autograd", autograd(pre.cpu(), g.cpu()).cuda()),
                  ("gpu emul", emul(pre, g)), ("cpu emul", emul(pre.cpu(), g.cpu()).cuda())):
    d = (dg.float() - ref).abs()
    print(f"{name:13s} exact {(d == 0).float().mean().item():.4f}  max {d.max().item():.3e}", flush=True)
ga, ge = autograd(pre, g), emul(pre, g)
print("gpu autograd vs gpu emul exact", ((ga - ge).abs() == 0).float().mean().item())
