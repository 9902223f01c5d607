"""Fused Adam / AdamW over the flat parameter buffer (K13/K14) and the HF LR
schedules the reference recipes name (transformers.get_scheduler semantics:
`cosine_with_min_lr` for Pythia, src/models/pythia.py:70-78; `cosine` for
llava-pretrain, src/models/llava.py:112-119).

One kernel launch updates every parameter of the (shard of the) model:
reads p32, g, m, v; writes p32, m, v and the bf16 shadow (28 B/param).
Gradient clipping (src/benchmarking/utils.py:66-70 → clip_grad_norm_) is a
deterministic Σg² reduction plus a device-side coefficient — no host sync.
"""

from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from . import kernels as K


@dataclass
class AdamConfig:
    lr: float = 1e-3
    betas: tuple[float, float] = (0.9, 0.999)
    eps: float = 1e-8
    weight_decay: float = 0.0
    adamw: bool = True
    max_grad_norm: float = 0.0


class FusedAdam:
    """Adam(W) on a flat fp32 buffer (or a ZeRO shard of it)."""

    def __init__(self, params: torch.Tensor, grads: torch.Tensor, shadow: torch.Tensor | None,
                 cfg: AdamConfig):
        if params.numel() % 4:
            raise ValueError("flat buffer length must be a multiple of 4")
        self.p, self.g, self.shadow, self.cfg = params, grads, shadow, cfg
        self.m = torch.zeros_like(params)
        self.v = torch.zeros_like(params)
        self.step_count = 0
        self._sumsq = torch.zeros(1, dtype=torch.float32, device=params.device)
        self._coef = torch.ones(1, dtype=torch.float32, device=params.device)

    def grad_sumsq(self) -> torch.Tensor:
        K.sumsq_f32(self.g, self._sumsq)
        return self._sumsq

    def step(self, lr: float, sumsq: torch.Tensor | None = None) -> None:
        """sumsq: global Σg² (already all-reduced under ZeRO); computed locally if None."""
        c = self.cfg
        self.step_count += 1
        scale = None
        if c.max_grad_norm and c.max_grad_norm > 0:
            if sumsq is None:
                sumsq = self.grad_sumsq()
            K.clip_coef(sumsq, c.max_grad_norm, self._coef)
            scale = self._coef
        K.adam_step(self.p, self.g, self.m, self.v, self.shadow, lr=lr, beta1=c.betas[0],
                    beta2=c.betas[1], eps=c.eps, weight_decay=c.weight_decay, adamw=c.adamw,
                    step=self.step_count, grad_scale=scale)

    def state_dict(self) -> dict:
        return {"m": self.m, "v": self.v, "step": self.step_count}


# ------------------------------------------------------------------ LR schedules
def lr_lambda(kind: str, step: int, num_warmup: int, num_training: int,
              min_lr_rate: float = 0.0) -> float:
    """transformers.optimization schedule multipliers (the value LambdaLR applies
    at optimizer step `step`, 0-based)."""
    if kind == "constant":
        return 1.0
    if step < num_warmup:
        return float(step) / float(max(1, num_warmup))
    if kind == "constant_with_warmup":
        return 1.0
    progress = float(step - num_warmup) / float(max(1, num_training - num_warmup))
    if kind == "linear":
        return max(0.0, 1.0 - progress)
    if kind == "cosine":
        return max(0.0, 0.5 * (1.0 + math.cos(math.pi * 0.5 * 2.0 * progress)))
    if kind == "cosine_with_min_lr":
        f = 0.5 * (1.0 + math.cos(math.pi * 0.5 * 2.0 * progress))
        return f * (1 - min_lr_rate) + min_lr_rate
    raise ValueError(f"unsupported scheduler {kind!r}")


class Schedule:
    def __init__(self, base_lr: float, kind: str, num_warmup_steps: int, num_training_steps: int,
                 min_lr_rate: float = 0.0):
        self.base_lr, self.kind = base_lr, kind
        self.warm, self.total, self.min_rate = num_warmup_steps, num_training_steps, min_lr_rate
        self.step_idx = 0

    def lr(self) -> float:
        return self.base_lr * lr_lambda(self.kind, self.step_idx, self.warm, self.total, self.min_rate)

    def step(self) -> None:
        self.step_idx += 1
