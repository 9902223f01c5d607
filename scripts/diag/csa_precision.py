"""Precision of the weight-gradient GEMM's row sums (EPI_F32_ACC_COLSUM) against fp64, beside
the column-sum kernel's: the fp32 partial rows summed in fp64 (before the bf16 rounding), on
positive data (a truncating accumulate would show as a one-sided error).  Diagnostic only."""
import json
import sys

import torch

sys.path.insert(0, ".")
from multimodal_llm_pretraining_amd import _lib, kernels as K  # noqa: E402

dev = "cuda"
for M, N, Kd in [(6144, 2048, 45248), (2048, 2048, 147456)]:
    torch.manual_seed(0)
    dY = torch.randn(Kd, M, device=dev).abs().to(torch.bfloat16)
    X = torch.randn(Kd, N, device=dev).to(torch.bfloat16)
    rows = _lib.query("mmpt_gemm_acc_colsum_rows", M, N, Kd)
    part = torch.zeros(rows, M, device=dev)
    G = torch.zeros(M, N, device=dev)
    K.gemm(dY, X, G, layout_a=K.K_ROWS, layout_b=K.K_ROWS, epilogue=K.EPI_F32_ACC_COLSUM, out2=part)
    ref = dY.double().sum(0)
    fused = part.double().sum(0)
    ws = K.workspace(_lib.query("mmpt_colsum_workspace_bytes", Kd, M), slot=1)
    _lib.call("mmpt_colsum_bf16", Kd, M, dY.data_ptr(), M, part.data_ptr(), None, 0, ws.data_ptr(),
              torch.cuda.current_stream().cuda_stream)  # (stage-2 output only: row 0 of part)
    torch.cuda.synchronize()
    nch = (Kd + 127) // 128
    stage1 = ws[: nch * M * 4].view(torch.float32).view(nch, M).double().sum(0)
    for name, v in (("fused", fused), ("colsum", stage1)):
        rel = (v - ref) / ref
        print(json.dumps({"M": M, "K": Kd, "form": name, "rows": rows if name == "fused" else nch,
                          "mean_rel": rel.mean().item(), "max_abs_rel": rel.abs().max().item()}))
