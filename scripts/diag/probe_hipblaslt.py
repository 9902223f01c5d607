"""Probe (diagnostic only, not on the product path): which hipBLASLt kernels torch.matmul
picks for the step's GEMM shapes, and how fast they run, next to libmmpt's GEMM."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from multimodal_llm_pretraining_amd import kernels as K  # noqa: E402

shapes = [(45248, 8192, 2048), (45248, 2048, 8192), (45248, 6144, 2048), (45248, 2048, 2048),
          (8192, 8192, 8192)]
for M, N, Kd in shapes:
    a = torch.randn(M, Kd, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, Kd, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for name, fn in (("hipblaslt", lambda: torch.matmul(a, b.t(), out=out)),
                     ("mmpt", lambda: K.gemm(a, b, out))):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        print(f"{name:10s} {M}x{N}x{Kd}: {ms*1e3:8.1f} us  {2*M*N*Kd/ms/1e9:7.1f} TF/s", flush=True)
