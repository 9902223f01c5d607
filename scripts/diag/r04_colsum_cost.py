"""Diagnostic (wrong gradients, never a bench line): what the step would gain without the qkv
bias column sums (16 x 431 us per step, on the weight-gradient stream) — bench.py with
kernels.colsum turned into a no-op for 6144-column inputs (Pythia-1B's fused qkv), run beside
an unpatched bench on the same box (scripts/diag/r04_colsum_cost.sh)."""

import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from multimodal_llm_pretraining_amd import kernels as K  # noqa: E402

_orig = K.colsum


def _skip_qkv(dy, dbias, accumulate=True, dbias2=None):
    if dy.shape[1] == 6144:
        return None
    return _orig(dy, dbias, accumulate=accumulate, dbias2=dbias2)


K.colsum = _skip_qkv
sys.argv = ["bench.py"] + sys.argv[1:]
runpy.run_path("bench.py", run_name="__main__")
