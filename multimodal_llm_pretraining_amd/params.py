"""Flat parameter / gradient / optimizer-state storage in HBM.

Every parameter is a view into ONE flat fp32 master buffer, ONE bf16 shadow
buffer (the autocast weight copy, refreshed by the fused Adam kernel — K15:
no per-micro-step cast kernels) and ONE fp32 gradient buffer.  Offsets are
aligned to 64 elements (256 B fp32 / 128 B bf16) so every view satisfies the
16-B DMA alignment of the GEMM kernels, and the total is padded so the buffer
splits into `world` equal, aligned shards for ZeRO.
"""

from __future__ import annotations

import math
import os

import torch

ALIGN = 64


def is_fp32_read(name: str) -> bool:
    """Parameters the step reads from the fp32 MASTER (not the bf16 shadow): LayerNorm
    γ/β (fp32 under autocast), the token-embedding table (embedding lookups are not
    autocast) and the ViT CLS / position embeddings.  They are laid out first, in one
    contiguous region, so ZeRO can re-broadcast exactly that region after the update."""
    return name in ("text.embed", "vision.pos", "vision.cls") or ".ln" in name \
        or "final_ln" in name


class ParamStore:
    def __init__(self, shapes: dict[str, tuple[int, ...]], device: torch.device | str,
                 world: int = 1, grads: bool = True, trainable=None):
        """trainable: predicate of the parameters a partly frozen model trains
        (ModelConfig.trainable under freeze_tower_and_llm).  They must be contiguous in the
        layout; the range is started and ended on a multiple of ALIGN·world elements so
        the optimizer / gradient exchange over it (whole, equal, aligned shards) never
        touches a frozen parameter."""
        self.shapes = dict(shapes)
        self.device = torch.device(device)
        self.offsets: dict[str, int] = {}
        off = 0
        order = [n for n in self.shapes if is_fp32_read(n)] + \
            [n for n in self.shapes if not is_fp32_read(n)]
        tr = [n for n in order if trainable(n)] if trainable is not None else []
        if tr and len(tr) < len(order):
            first, last = order.index(tr[0]), order.index(tr[-1])
            if last - first + 1 != len(tr):
                raise RuntimeError("trainable parameters are not contiguous in the flat layout")
        for name in order:
            if tr and name == tr[0]:
                off = _round(off, ALIGN * world)
            self.offsets[name] = off
            off += _round(math.prod(self.shapes[name]), ALIGN)
            if tr and name == tr[-1]:
                off = _round(off, ALIGN * world)
            if is_fp32_read(name):
                self.fp32_end = off
        self.fp32_end = getattr(self, "fp32_end", 0)  # [0, fp32_end): read as fp32
        self.numel = off
        self.world = world
        self.padded = _round(off, ALIGN * world)
        self.shard_size = self.padded // world
        self.master = torch.zeros(self.padded, dtype=torch.float32, device=self.device)
        self.shadow = torch.zeros(self.padded, dtype=torch.bfloat16, device=self.device)
        self.grad = torch.zeros(self.padded, dtype=torch.float32, device=self.device) if grads else None
        # transposed bf16 shadow of the GEMM weights (dX = dY·W reads W^T K-contiguous)
        self.shadow_t = torch.zeros(self.padded, dtype=torch.bfloat16, device=self.device)
        self.transposed: list[str] = []

    def names(self):
        return list(self.shapes)

    def _view(self, buf: torch.Tensor, name: str) -> torch.Tensor:
        o = self.offsets[name]
        shape = self.shapes[name]
        return buf[o:o + math.prod(shape)].view(shape)

    def p(self, name: str) -> torch.Tensor:
        """fp32 master view (after release_master: a host view outside the kept region)"""
        o = self.offsets[name]
        if self.host_master is not None and o >= self.master.numel():
            lo = o - self.host_lo
            n = math.prod(self.shapes[name])
            if lo < 0 or lo + n > self.host_master.numel():
                raise RuntimeError(f"{name}: its fp32 master lives on another rank's host")
            return self.host_master[lo:lo + n].view(self.shapes[name])
        return self._view(self.master, name)

    # ---- optimizer offload (DeepSpeed offload_optimizer, src/train.py:203-207): the fp32
    # master moves to host memory; the device keeps only the region the step reads as fp32
    host_master: torch.Tensor | None = None
    host_lo = 0

    def release_master(self, keep: int, host: torch.Tensor, host_lo: int) -> torch.Tensor:
        """Drop the device fp32 master past `keep` elements (the fp32-read region, which the
        step reads on the device); `host` (fp32, this rank's optimizer range starting at
        flat offset host_lo) is the authoritative copy from now on.  Returns the new, small
        device master."""
        self.master = self.master[:keep].clone()
        self.host_master, self.host_lo = host, host_lo
        return self.master

    def restore_master(self) -> torch.Tensor:
        """Re-materialise the full device master from the host copy (checkpoints, tests);
        outside this rank's host range the values are the kept region or zero."""
        if self.host_master is None:
            return self.master
        full = torch.zeros(self.padded, dtype=torch.float32, device=self.device)
        full[:self.master.numel()].copy_(self.master)
        h = self.host_master
        full[self.host_lo:self.host_lo + h.numel()].copy_(h, non_blocking=False)
        self.master, self.host_master, self.host_lo = full, None, 0
        return full

    def w(self, name: str) -> torch.Tensor:
        """bf16 shadow view (GEMM operand)"""
        return self._view(self.shadow, name)

    def wt(self, name: str) -> torch.Tensor:
        """bf16 transposed shadow view [in, out] of a 2-D weight [out, in]"""
        o = self.offsets[name]
        r, c = self.shapes[name]
        return self.shadow_t[o:o + r * c].view(c, r)

    def g(self, name: str) -> torch.Tensor:
        """fp32 gradient view"""
        return self._view(self.grad, name)

    def shard(self, buf: torch.Tensor, rank: int) -> torch.Tensor:
        return buf[rank * self.shard_size:(rank + 1) * self.shard_size]

    def load(self, tensors: dict[str, torch.Tensor]) -> None:
        """Copy full tensors into the fp32 master (after release_master: the host copy,
        and for the kept region both copies)."""
        for name, t in tensors.items():
            if self.host_master is not None:
                # this rank's host range may cut through the parameter (ZeRO-1 shards are
                # padded/world elements, not parameter-aligned): copy the overlap
                o, n = self.offsets[name], math.prod(self.shapes[name])
                h_lo, h_hi = self.host_lo, self.host_lo + self.host_master.numel()
                lo, hi = max(o, h_lo), min(o + n, h_hi)
                if lo < hi:
                    flat = t.reshape(-1).to("cpu", torch.float32)
                    self.host_master[lo - h_lo:hi - h_lo].copy_(flat[lo - o:hi - o])
                # the replicated bf16 shadow: refresh_shadow can only re-cast this rank's
                # host range, so the whole tensor (every rank loads all of it) goes in here
                self.w(name).copy_(t.to(self.device, torch.float32).to(torch.bfloat16))
                if o >= self.master.numel():
                    continue
            self.p(name).copy_(t.to(self.device, torch.float32))

    def state_dict(self) -> dict[str, torch.Tensor]:
        return {n: self.p(n).detach().clone() for n in self.shapes}

    def refresh_shadow(self) -> None:
        from . import kernels as K

        K.cast_f32_bf16(self.master, self.shadow[:self.master.numel()])
        if self.host_master is not None:  # released master: the rest from the host copy
            keep, h = self.master.numel(), self.host_master
            lo = max(keep, self.host_lo)
            if lo < self.host_lo + h.numel():
                self.shadow[lo:self.host_lo + h.numel()].copy_(
                    h[lo - self.host_lo:].to(torch.bfloat16))
        self.refresh_transposed()

    def refresh_transposed(self, names: list[str] | None = None) -> None:
        """Rebuild W^T for `names` (default: every transposed weight) — on the device in one
        launch (mmpt_transpose_bf16_batched, descriptors cached per name list), else one
        transpose per weight."""
        from . import kernels as K

        names = list(self.transposed if names is None else names)
        if not names:
            return
        if self.device.type != "cuda" or os.environ.get("MMPT_WT_BATCHED", "1") == "0":
            for name in names:
                K.transpose_bf16(self.w(name), self.wt(name))
            return
        key = tuple(names)
        cache = self.__dict__.setdefault("_wt_desc", {})
        if key not in cache:
            rows, tiles = [], 0
            for name in names:
                r, c = self.shapes[name]
                rows.append((self.offsets[name], r, c, tiles))
                tiles += ((r + 63) // 64) * ((c + 63) // 64)
            cache[key] = (torch.tensor(rows, dtype=torch.int64, device=self.device), tiles)
        desc, tiles = cache[key]
        K.transpose_bf16_batched(self.shadow, self.shadow_t, desc, tiles)

    def zero_grad(self) -> None:
        if self.grad is not None:
            self.grad.zero_()


def _round(n: int, m: int) -> int:
    return (n + m - 1) // m * m


def init_normal(store: ParamStore, seed: int = 0, std: float = 0.02, cfg=None) -> None:
    """Deterministic random init (weights N(0, std), LN gains 1, biases N(0, std)) —
    generated on the CPU so every rank / the oracle see identical bits."""
    g = torch.Generator().manual_seed(seed)
    for name, shape in store.shapes.items():
        if name.endswith(("ln1.weight", "ln2.weight", "final_ln.weight", "ln_pre.weight")):
            t = torch.ones(shape)
        else:
            t = torch.randn(shape, generator=g) * std
        if name == "vision.patch.weight" and cfg is not None:  # im2col pad columns stay 0
            v = cfg.vision
            t[:, v.channels * v.patch * v.patch:] = 0
        if name in ("text.embed", "text.lm_head") and cfg is not None:
            t[cfg.text.n_vocab:] = 0  # vocabulary padding rows (never read, zero gradient)
        store.load({name: t})
    store.refresh_shadow()
