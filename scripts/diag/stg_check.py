"""Diagnostic: the plain gemm4p result of this library vs a reference library build (MMPT_REF_LIB,
loaded in a child process) on the same seeded operands; prints mismatch counts / locations."""
import os
import subprocess
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
shapes = [(4104, 4096, 320), (8192, 4096, 320), (4096, 2048, 2048), (65536, 2048, 512)]
out = sys.argv[1] if len(sys.argv) > 1 else None
from multimodal_llm_pretraining_amd import kernels as K  # noqa: E402

res = {}
for M, N, Kd in shapes:
    g = torch.Generator(device="cuda").manual_seed(5)
    A = torch.randn(M, Kd, device="cuda", generator=g).to(torch.bfloat16)
    W = torch.randn(N, Kd, device="cuda", generator=g).to(torch.bfloat16)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    K.gemm(A, W, c)
    torch.cuda.synchronize()
    res[(M, N, Kd)] = c.cpu()
if out:
    torch.save(res, out)
    sys.exit(0)
ref_path = "/tmp/stg_ref.pt"
env = dict(os.environ, MMPT_LIB=os.environ["MMPT_REF_LIB"])
subprocess.run([sys.executable, __file__, ref_path], env=env, check=True)
ref = torch.load(ref_path)
for k, v in res.items():
    d = (v.view(torch.int16) != ref[k].view(torch.int16))
    n = int(d.sum())
    print(k, "mismatches", n, flush=True)
    if n:
        idx = d.nonzero()
        rows, cols = idx[:, 0], idx[:, 1]
        print("  rows tiles:", sorted(set((rows // 256).tolist()))[:20], "cols tiles:", sorted(set((cols // 256).tolist()))[:20])
        print("  row%256 range", int((rows % 256).min()), int((rows % 256).max()), "col%256 range", int((cols % 256).min()), int((cols % 256).max()))
