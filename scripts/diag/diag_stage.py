"""Where does the GELU act output of the staged epilogue disagree with GELU(pre)?"""
import torch
from multimodal_llm_pretraining_amd import kernels as K

dev = "cuda"
torch.manual_seed(41 + 256)
M, N, Kd = 20232, 4096, 256
bf = lambda t: t.to(torch.bfloat16)
A = bf(torch.randn(M, Kd, device=dev))
W = bf(torch.randn(N, Kd, device=dev) * 0.05)
bias = bf(torch.randn(N, device=dev))
pre = torch.full((M, N), 7.0, device=dev, dtype=torch.bfloat16)
act = torch.full((M, N), 7.0, device=dev, dtype=torch.bfloat16)
K.gemm(A, W, pre, epilogue=K.EPI_BF16_GELU, bias=bias, out2=act)
want = torch.nn.functional.gelu(pre.float()).to(torch.bfloat16)
ulp = (act.view(torch.int16).int() - want.view(torch.int16).int()).abs()
bad = ulp > 1
print("bad", int(bad.sum()), "of", M * N, "unwritten act", int((act == 7.0).sum()), "unwritten pre", int((pre == 7.0).sum()))
idx = bad.nonzero()[:20].tolist()
for r, c in idx:
    print(r, c, "tile", r // 256, c // 256, "pre", pre[r, c].item(), "act", act[r, c].item(), "want", want[r, c].item())
rows = bad.any(1).nonzero().flatten()
cols = bad.any(0).nonzero().flatten()
print("bad rows", rows.numel(), rows[:20].tolist(), "bad cols", cols.numel(), cols[:20].tolist())
