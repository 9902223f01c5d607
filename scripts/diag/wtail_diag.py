"""Where does the weight-gradient tail split differ from the fp32 product (debug helper)."""
import sys

import torch

sys.path.insert(0, ".")
from multimodal_llm_pretraining_amd import _lib  # noqa: E402
from multimodal_llm_pretraining_amd import kernels as K  # noqa: E402

dev = "cuda"
for (M, N, Kd, mode) in [(5120, 3328, 8192, 1), (3328, 5120, 8192, 2)]:
    torch.manual_seed(23)
    a = torch.randn(Kd, M, device=dev).to(torch.bfloat16)
    b = torch.randn(Kd, N, device=dev).to(torch.bfloat16)
    c0 = torch.randn(M, N, device=dev)
    prod = a.float().t() @ b.float()
    want = prod.to(torch.bfloat16).float() + c0
    for w in (0, mode):
        _lib.set_switch("MMPT_GEMM_WTAIL", w)
        c = c0.clone()
        K.gemm(a, b, c, layout_a=K.K_ROWS, layout_b=K.K_ROWS, epilogue=K.EPI_F32_ACC)
        torch.cuda.synchronize()
        d = (c - want).abs()
        lim = 2.0 ** -8 * prod.abs() + 1e-5 * want.abs() + 1e-3
        bad = d > lim
        print(M, N, Kd, "wtail", w, K.gemm_last_kernel(), "bad", int(bad.sum()), "max", float(d.max()),
              flush=True)
        if bad.any():
            r, q = torch.nonzero(bad, as_tuple=True)
            print("  rows", int(r.min()), int(r.max()), "cols", int(q.min()), int(q.max()),
                  "sample", [(int(r[i]), int(q[i]), float(c[r[i], q[i]]), float(want[r[i], q[i]]))
                             for i in range(min(4, len(r)))], flush=True)
            print("  ratio d/prod at bad", float((d[bad] / prod.abs()[bad].clamp_min(1e-6)).max()), flush=True)
