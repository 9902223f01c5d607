"""GPU table (src/gpus.py), extended with the MI355X.

`ampere_or_newer_gpu` keeps its role in the reference: it gates bf16 recipes
(training_time_empirical.py:170) and turns tf32 on for free_lunch
(experiments/config.py:43-45).  On the MI355X bf16 is native, while the tf32 flag
(torch.backends.cuda.matmul.allow_tf32) has nothing to act on — every GEMM of the
path is an explicit bf16 MFMA kernel — so `tf32_capable` is False for it.
"""

from __future__ import annotations

from typing import Literal

GpuT = Literal["geforce3090", "v100", "a6000", "a40", "l40", "a100", "h100", "mi355x"]
GPUS = ("geforce3090", "v100", "a6000", "a40", "l40", "a100", "h100", "mi355x")


def ampere_or_newer_gpu(gpu_type: str) -> bool:
    if gpu_type not in GPUS:
        raise ValueError(f"unknown gpu type {gpu_type!r}")
    return gpu_type != "v100"


def tf32_capable(gpu_type: str) -> bool:
    return ampere_or_newer_gpu(gpu_type) and gpu_type != "mi355x"
