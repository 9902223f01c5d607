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
import os
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

    def step(self, lr: float, sumsq: torch.Tensor | None = None, zero_grad: bool = False) -> None:
        """sumsq: global Σg² (already all-reduced under ZeRO); computed locally if None.
        zero_grad: the update also zeroes the gradient it consumes (one pass less)."""
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
                    step=self.step_count, grad_scale=scale, zero_grad=zero_grad)

    def state_dict(self) -> dict:
        return {"m": self.m, "v": self.v, "step": self.step_count}


class AdamOverlap:
    """The optimizer step overlapped with the next step's forward (round 6).

    For the flat store of the data-parallel / single-GPU step (ParamStore + FusedAdam over the
    whole buffer): instead of one Adam launch, a zero_grad pass and the W^T refresh on the
    compute stream between two steps, `step` queues them per parameter unit on an optimizer
    stream — the fp32-read region (embeddings, LayerNorms) first, then the units in forward
    order (vision patch, vision layers, projector, text layers, lm_head) — and the next forward
    waits for a unit's update right before it first reads that unit (this object is the
    engine's `units` hook, as offload.OffloadGate is for the host update).  Same arithmetic as
    FusedAdam.step on the same values: bitwise the serial step.

    Measured (round 6, 32 samples per rank, one box, 6-step lines): 248.9 samples/s overlapped
    (256-workgroup updates) vs 252.1 serial, 252.3 with full-grid updates, 245.3 with 128
    workgroups — the 33 GB of update traffic slows the forward's GEMMs as much as it saves, so
    it is OFF by default (MMPT_ADAM_OVERLAP=1 turns it on); the serial step keeps the fused
    zero_grad (mmpt_adam_step_zero_grad).
    Clipping (when configured) still needs the global gradient norm first: Σg² and the clip
    coefficient run on the compute stream, the per-unit updates read the coefficient."""

    def __init__(self, store, opt: FusedAdam, order: list[str]):
        from .zero3 import unit_of

        self.s, self.opt = store, opt
        self.dev = store.device
        self.stream = torch.cuda.Stream(device=self.dev)
        ranges: dict[str, list[int]] = {}
        self.trans: dict[str | None, list[str]] = {}
        for n, o in store.offsets.items():
            try:
                u = unit_of(n)
            except KeyError:
                u = None
            if u is None:
                if o >= store.fp32_end:
                    raise RuntimeError(f"{n}: outside the fp32-read region and without a unit")
            else:
                r = ranges.setdefault(u, [o, o + store.g(n).numel()])
                r[0], r[1] = min(r[0], o), max(r[1], o + store.g(n).numel())
            if n in store.transposed:
                self.trans.setdefault(u, []).append(n)
        missing = set(ranges) - set(order)
        if missing:
            raise RuntimeError(f"units outside the forward order: {sorted(missing)}")
        # the region, then the units in forward order (the alignment gaps between parameters
        # and the padding tail hold zeros with zero gradients: an update leaves them zero)
        self.chunks: list[tuple[str | None, int, int]] = [(None, 0, store.fp32_end)]
        self.chunks += [(u, ranges[u][0], ranges[u][1]) for u in order if u in ranges]
        cover = sorted((lo, hi) for _, lo, hi in self.chunks)
        pos = 0
        for lo, hi in cover:
            if lo < pos:
                raise RuntimeError("parameter units overlap in the flat layout")
            pos = hi
        self.fwd: dict[str | None, torch.cuda.Event] = {}
        self.bwd: dict[str | None, torch.cuda.Event] = {}
        self.pending_f: set = set()
        self.pending_b: set = set()
        # workgroups of each update launch (MMPT_ADAM_BLOCKS; 0 = the serial kernel's grid)
        self.max_blocks = int(os.environ.get("MMPT_ADAM_BLOCKS", "0"))

    def step(self, lr: float, sumsq: torch.Tensor | None = None) -> None:
        from . import kernels as K

        o, c = self.opt, self.opt.cfg
        o.step_count += 1
        scale = None
        if c.max_grad_norm and c.max_grad_norm > 0:
            if sumsq is None:
                sumsq = o.grad_sumsq()
            K.clip_coef(sumsq, c.max_grad_norm, o._coef)
            scale = o._coef
        cur = torch.cuda.current_stream(self.dev)
        self.stream.wait_stream(cur)  # after the backward (and the gradient exchange)
        with torch.cuda.stream(self.stream):
            # the updates in forward order, then the W^T refreshes: the forward reads a unit's
            # bf16 weights (event `fwd`), only its backward reads the transposes (event `bwd`)
            for u, lo, hi in self.chunks:
                if hi <= lo:
                    continue
                K.adam_step(o.p[lo:hi], o.g[lo:hi], o.m[lo:hi], o.v[lo:hi],
                            None if o.shadow is None else o.shadow[lo:hi], lr=lr,
                            beta1=c.betas[0], beta2=c.betas[1], eps=c.eps,
                            weight_decay=c.weight_decay, adamw=c.adamw, step=o.step_count,
                            grad_scale=scale, zero_grad=True, max_blocks=self.max_blocks)
                self.fwd[u] = torch.cuda.Event()
                self.fwd[u].record(self.stream)
            end = max(hi for _, _, hi in self.chunks)
            if end < o.g.numel():  # the padding tail (zero parameters and gradients)
                o.g[end:].zero_()
            for u, lo, hi in self.chunks:
                for n in self.trans.get(u, []):
                    K.transpose_bf16(self.s.w(n), self.s.wt(n))
                self.bwd[u] = torch.cuda.Event()
                self.bwd[u].record(self.stream)
        self.pending_f = {u for u, lo, hi in self.chunks if hi > lo}
        self.pending_b = {u for u, _, _ in self.chunks}

    def _wait(self, pending: set, events: dict, u) -> None:
        if u in pending:
            torch.cuda.current_stream(self.dev).wait_event(events[u])
            pending.discard(u)

    # ---- the engine's `units` hook
    def region(self) -> None:
        """Before a forward: the fp32-read region's update is in."""
        self._wait(self.pending_f, self.fwd, None)

    def forward(self, unit: str) -> None:
        self._wait(self.pending_f, self.fwd, unit)

    def backward(self, unit: str) -> None:
        """Before a unit's backward: its update and W^T (and the region's: a tied lm_head's
        input gradient reads E^T) are in."""
        self._wait(self.pending_f, self.fwd, unit)
        self._wait(self.pending_b, self.bwd, None)
        self._wait(self.pending_b, self.bwd, unit)

    def backward_done(self, unit: str) -> None:
        pass

    def open_grad(self, unit: str) -> None:
        pass

    def join(self) -> None:
        """Every update is in: the compute stream is ordered after the optimizer stream."""
        if self.pending_f or self.pending_b:
            torch.cuda.current_stream(self.dev).wait_stream(self.stream)
            self.pending_f, self.pending_b = set(), set()

    def reset(self) -> None:
        self.join()


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
