"""Diagnostic (GPU): the gemm4p quick-GELU / SwiGLU forms on every finite bf16 input against
torch's CPU bf16 ops — prints every mismatch class instead of stopping at the first (the test
is tests/test_kernels_gpu.py::test_gemm4p_activation_tables_every_bf16_input)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from multimodal_llm_pretraining_amd import kernels as K  # noqa: E402

dev = "cuda"


def report(tag, got, want, xs, other):
    g, w = got.float().cpu(), want.float().cpu()
    both_nan = torch.isnan(g) & torch.isnan(w)
    diff = (g != w) & ~both_nan
    tiny = (g.abs() < 1e-37) & (w.abs() < 1e-37)
    big = diff & ~tiny
    print(tag, "kernel", K.gemm_last_kernel(), "diff", int(diff.sum()), "non-tiny", int(big.sum()))
    for i in big.nonzero().flatten()[:12].tolist():
        print(f"   x={xs[i].item()!r} other={other[i].item()!r} got={g[i].item()!r} want={w[i].item()!r}")


def main():
    M = 65536
    bits = torch.arange(0, 1 << 16, dtype=torch.int32).to(torch.int16)
    xs = bits.view(torch.bfloat16).float()
    xs = xs[torch.isfinite(xs)]
    xs = xs.repeat(-(-M // xs.numel()))[:M].to(torch.bfloat16)
    torch.manual_seed(31)
    other = (torch.randn(M) * 2).to(torch.bfloat16)
    A = torch.zeros(M, 64, dtype=torch.bfloat16)
    A[:, 0] = xs
    A[:, 1] = other
    A = A.to(dev)
    W = torch.zeros(256, 64, device=dev, dtype=torch.bfloat16)
    W[0, 0] = 1.0
    pre = torch.empty(M, 256, device=dev, dtype=torch.bfloat16)
    act = torch.empty_like(pre)
    K.gemm(A, W, pre, epilogue=K.EPI_BF16_QGELU, out2=act)
    report("qgelu", act[:, 0], xs * torch.sigmoid(1.702 * xs), xs, other)
    W2 = torch.zeros(256, 64, device=dev, dtype=torch.bfloat16)
    W2[0, 1] = 1.0
    dg = torch.empty_like(pre)
    K.gemm(A, W2, dg, epilogue=K.EPI_BF16_DQGELU, aux=pre)
    x = xs.clone().requires_grad_()
    (x * torch.sigmoid(1.702 * x)).backward(other)
    report("dqgelu", dg[:, 0], x.grad, xs, other)
    Wg = torch.zeros(256, 64, device=dev, dtype=torch.bfloat16)
    Wg[0, 0] = 1.0
    Wg[128, 1] = 1.0
    gu = torch.empty(M, 256, device=dev, dtype=torch.bfloat16)
    sact = torch.empty(M, 128, device=dev, dtype=torch.bfloat16)
    K.gemm(A, Wg, gu, epilogue=K.EPI_BF16_SWIGLU, out2=sact)
    print("gu gate/up exact:", torch.equal(gu[:, 0].cpu(), xs), torch.equal(gu[:, 128].cpu(), other),
          "zeros elsewhere:", not gu[:, 1:128].cpu().any(), not sact[:, 1:].cpu().any())
    report("swiglu", sact[:, 0], torch.nn.functional.silu(xs) * other, xs, other)
    wdt = torch.zeros(128, 64, device=dev, dtype=torch.bfloat16)
    wdt[0, 1] = 1.0
    dgu = torch.empty(M, 256, device=dev, dtype=torch.bfloat16)
    K.gemm(A, wdt, dgu, epilogue=K.EPI_BF16_DSWIGLU, aux=gu)
    gr, ur = xs.clone().requires_grad_(), other.clone().requires_grad_()
    (torch.nn.functional.silu(gr) * ur).backward(other)
    report("dswiglu gate", dgu[:, 0], gr.grad, xs, other)
    report("dswiglu up", dgu[:, 128], ur.grad, xs, other)


if __name__ == "__main__":
    main()
