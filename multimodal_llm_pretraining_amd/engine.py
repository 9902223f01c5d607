"""Forward / backward of one micro-batch of the ViT → projector → Pythia step,
written explicitly over the libmmpt HIP kernels (no torch.autograd on the hot
path, no ATen compute).

Mirrors, op for op, the arithmetic HF runs inside
`Trainer.training_step` → `model(**inputs).loss` → `backward()` for
LlavaForConditionalGeneration(ViT, GPTNeoX) / GPTNeoXForCausalLM under bf16
autocast (reference call stack: SURVEY.md §3.2; math:
tf:models/gpt_neox/modeling_gpt_neox.py:180-384, tf:models/vit/modeling_vit.py:
42-300, tf:models/llava/modeling_llava.py:87-248, tf:loss/loss_utils.py:32-68):

* residual streams fp32, LayerNorm fp32 → bf16 GEMM operand (fused cast);
* GEMMs bf16 × bf16 → fp32 accumulate → bf16 out, bias/GELU/residual fused in
  the epilogue; weight grads rounded to bf16 then accumulated in fp32
  (autocast's bf16 grad → fp32 .grad);
* attention via the flash kernels, partial RoPE in place on the fused qkv;
* cross-entropy fused fwd+bwd over bf16 logits (fp32 math), dlogits in place.
"""

from __future__ import annotations

import os

import numpy as np
import torch

from . import kernels as K
from .config import ModelConfig
from .params import ParamStore

BF16 = torch.bfloat16
F32 = torch.float32


def rope_tables(hidden: int, heads: int, rotary_pct: float, theta: float, seq: int):
    """cos/sin [seq][rot] in fp32, computed on the CPU exactly as
    tf:modeling_gpt_neox.py:76-110 does (so the oracle and the GPU share bits)."""
    head_dim = hidden // heads
    dim = int(head_dim * rotary_pct)
    inv_freq = 1.0 / (theta ** (torch.arange(0, dim, 2, dtype=torch.int64).float() / dim))
    pos = torch.arange(seq).float()
    freqs = pos[:, None] * inv_freq[None, :]
    emb = torch.cat((freqs, freqs), dim=-1)
    return emb.cos().contiguous(), emb.sin().contiguous()


def rope_tables_llama3(head_dim: int, theta: float, scaling, seq: int):
    """Llama-3 rotary tables (transformers modeling_rope_utils.py _compute_llama3_parameters:
    inverse frequencies rescaled by `factor` below the low-frequency wavelength and smoothly
    interpolated in between; LlamaRotaryEmbedding.forward: fp32 outer product, cat, cos/sin,
    attention factor 1), computed on the CPU with HF's own op sequence."""
    import math

    inv_freq = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.int64).float() / head_dim))
    if scaling is not None:
        factor, low, high, old = scaling
        low_wl, high_wl = old / low, old / high
        wavelen = 2 * math.pi / inv_freq
        inv_l = torch.where(wavelen > low_wl, inv_freq / factor, inv_freq)
        smooth = (old / wavelen - low) / (high - low)
        smoothed = (1 - smooth) * inv_l / factor + smooth * inv_l
        medium = ~(wavelen < high_wl) * ~(wavelen > low_wl)
        inv_freq = torch.where(medium, smoothed, inv_l)
    pos = torch.arange(seq).float()
    with torch.autocast("cpu", enabled=False):
        freqs = (inv_freq[None, :, None] @ pos[None, None, :]).transpose(1, 2)[0]
        emb = torch.cat((freqs, freqs), dim=-1)
        return emb.cos().contiguous(), emb.sin().contiguous()


def sort_segments(ids: np.ndarray, rows: np.ndarray):
    """(seg_id, seg_off, perm) int32 for mmpt_embed_bwd: `rows` stably sorted by ids[row],
    one segment per distinct id (perm[seg_off[s]:seg_off[s+1]] all have id seg_id[s])."""
    perm = rows[np.argsort(ids[rows], kind="stable")]
    sid = ids[perm]
    starts = np.concatenate(([0], np.flatnonzero(np.diff(sid)) + 1)) if sid.size else \
        np.zeros(0, np.int64)
    seg_off = np.concatenate((starts, [perm.size]))
    return tuple(np.ascontiguousarray(a, dtype=np.int32) for a in (sid[starts], seg_off, perm))


class Batch:
    """A micro-batch staged in HBM with its index bookkeeping precomputed (label shift,
    loss-row compaction, image-token map, the embedding backward's id segments): the step
    reads only device memory.

    Host tensors (what a data loader yields, ideally pinned): the bookkeeping that sizes
    kernels (label count, scored rows, image-slot count) is computed from the host copy, the
    id segments are sorted on the device (`mmpt_embed_segments`), and every host-to-device
    copy is asynchronous on the current stream — building a Batch never waits for the GPU,
    so it can sit inside the timed step like the reference's `_prepare_inputs`
    (src/benchmarking/utils.py:61-63 → Trainer.training_step).  Device tensors are accepted
    too; the counts then cost one device synchronisation."""

    def __init__(self, cfg: ModelConfig, input_ids: torch.Tensor, labels: torch.Tensor,
                 pixel_values: torch.Tensor | None, device: torch.device, stream=None):
        """stream: stage on this (copy) stream instead of the current one — the copies and
        the segment sort then overlap the compute stream's work; `use(stream)` (called by
        Engine.forward) orders the consumer after them."""
        device = torch.device(device)
        self.B, self.S = input_ids.shape
        if cfg.multimodal and pixel_values is None:
            raise ValueError("multimodal model needs pixel_values")
        self._ready = None
        if stream is not None and device.type == "cuda":
            with torch.cuda.stream(stream):
                self._stage(cfg, input_ids, labels, pixel_values, device)
            self._ready = torch.cuda.Event()
            self._ready.record(stream)
        else:
            self._stage(cfg, input_ids, labels, pixel_values, device)

    def _stage(self, cfg, input_ids, labels, pixel_values, device):
        if input_ids.device.type == "cpu" and labels.device.type == "cpu":
            self._from_host(cfg, input_ids, labels, device)
        else:
            self._from_device(cfg, input_ids, labels, device)
        self.pixels = None
        if cfg.multimodal:
            self.pixels = _to(pixel_values, device, F32)
        self.segments = self._segments(cfg, input_ids, device)

    def use(self, stream) -> None:
        """Order `stream` after the staging stream and hand the staged tensors to it (the
        caching allocator then frees them only after `stream`'s use)."""
        if self._ready is None:
            return
        stream.wait_event(self._ready)
        for t in (self.ids, self.labels, self.loss_rows, self.loss_labels, self.loss_map,
                  self.img_map, self.pixels, *self.segments):
            if t is not None:
                t.record_stream(stream)
        self._ready = None

    def _from_host(self, cfg, input_ids, labels, device):
        ids = input_ids.reshape(-1).to(torch.int64)
        lab = labels.to(torch.int64)
        idn = ids.numpy()
        if idn.size and (idn.min() < 0 or idn.max() >= cfg.text.vocab):
            raise ValueError(f"token ids must lie in [0, {cfg.text.vocab})")
        shifted = torch.full_like(lab, -100)
        shifted[:, :-1] = lab[:, 1:]  # ForCausalLMLoss: pad(labels, (0,1)) then [..., 1:]
        shifted = shifted.reshape(-1)
        keep = (shifted != -100).numpy()
        _check_labels(shifted.numpy()[keep], cfg.text.n_vocab)
        self.num_items = int(keep.sum())
        self.ids = _to(ids, device, torch.int64)
        self.labels = _to(shifted, device, torch.int64)
        # loss-row compaction (mmpt_gather_rows_bf16): the lm_head / CE run over the rows
        # whose label is not ignored — for LLaVA batches the image-token rows (their logits
        # are never consumed; their gradient is exactly zero), e.g. 511 of 707 rows for
        # ViT-B/16 + 511 text tokens.  Text-only batches keep every row but the last.
        self.loss_rows = self.loss_map = None
        self.loss_labels = self.labels
        if self.num_items < 0.95 * keep.size:
            idx = np.flatnonzero(keep)
            lmap = np.full(keep.size, -1, np.int32)
            lmap[idx] = np.arange(idx.size, dtype=np.int32)
            self.loss_rows = _to(torch.from_numpy(idx.astype(np.int32)), device, torch.int32)
            self.loss_labels = _to(shifted[torch.from_numpy(idx)], device, torch.int64)
            self.loss_map = _to(torch.from_numpy(lmap), device, torch.int32)
        self.img_map = None
        if cfg.multimodal:
            mask = idn == cfg.image_token_id
            n_img = int(mask.sum())
            expect = self.B * cfg.vision.num_patches
            if n_img != expect:  # tf:modeling_llava.py get_placeholder_mask raises likewise
                raise ValueError(f"image tokens {n_img} != features {expect}")
            imap = np.where(mask, np.cumsum(mask) - 1, -1).astype(np.int32)
            self.img_map = _to(torch.from_numpy(imap), device, torch.int32)

    def _from_device(self, cfg, input_ids, labels, device):
        self.ids = input_ids.to(device, torch.int64).contiguous().view(-1)
        # the embedding kernels index the table without bounds checks: validate here (the
        # path synchronises for the counts below anyway)
        if self.ids.numel():
            lo_hi = torch.stack((self.ids.min(), self.ids.max())).tolist()
            if lo_hi[0] < 0 or lo_hi[1] >= cfg.text.vocab:
                raise ValueError(f"token ids must lie in [0, {cfg.text.vocab})")
        lab = labels.to(device, torch.int64)
        shifted = torch.full_like(lab, -100)
        shifted[:, :-1] = lab[:, 1:]
        self.labels = shifted.contiguous().view(-1)
        keep = self.labels != -100
        self.num_items = int(keep.sum().item())
        if self.num_items:
            kept = self.labels[keep]
            _check_labels(torch.stack((kept.min(), kept.max())).cpu().numpy(), cfg.text.n_vocab)
        self.loss_rows = self.loss_map = None
        self.loss_labels = self.labels
        if self.num_items < 0.95 * self.labels.numel():
            idx = torch.nonzero(keep).view(-1)
            self.loss_rows = idx.to(torch.int32).contiguous()
            self.loss_labels = self.labels[idx].contiguous()
            self.loss_map = torch.full_like(self.labels, -1, dtype=torch.int32)
            self.loss_map[idx] = torch.arange(idx.numel(), device=self.labels.device,
                                              dtype=torch.int32)
        self.img_map = None
        if cfg.multimodal:
            mask = self.ids == cfg.image_token_id
            n_img = int(mask.sum().item())
            expect = self.B * cfg.vision.num_patches
            if n_img != expect:
                raise ValueError(f"image tokens {n_img} != features {expect}")
            self.img_map = torch.where(mask, mask.cumsum(0) - 1, -1).to(torch.int32).contiguous()

    def _segments(self, cfg: ModelConfig, input_ids: torch.Tensor, device) -> tuple:
        """Index bookkeeping for the deterministic embedding backward: the
        text rows stably sorted by token id, one segment per distinct id — built on the
        device by `mmpt_embed_segments` (seg_id, seg_off, perm, nseg, bad), the count left in
        HBM.  (A CPU `device` — host-logic tests only, the engine cannot run there — uses
        the numpy restatement `sort_segments`.)"""
        skip = cfg.image_token_id if cfg.multimodal else -1
        if device.type != "cuda":
            ids = input_ids.reshape(-1).to("cpu", torch.int64).numpy()
            rows = np.arange(ids.size) if skip < 0 else np.flatnonzero(ids != skip)
            return tuple(torch.from_numpy(a) for a in sort_segments(ids, rows))
        return K.embed_segments(self.ids, cfg.text.vocab, skip)

    @property
    def tokens(self) -> int:
        return self.B * self.S


def _check_labels(kept: np.ndarray, vocab_valid: int) -> None:
    """Labels other than -100 must index a real vocabulary row (torch's nll_loss asserts on
    the device; the cross-entropy kernel would report NaN for the row)."""
    if kept.size and (kept.min() < 0 or kept.max() >= vocab_valid):
        raise ValueError(f"labels must be -100 or lie in [0, {vocab_valid})")


def _to(t: torch.Tensor, device: torch.device, dtype) -> torch.Tensor:
    """Asynchronous host-to-device staging (pinned when the loader pinned it)."""
    t = t.to(dtype).contiguous()
    if device.type == "cuda" and t.device.type == "cpu":
        return t.to(device, non_blocking=t.is_pinned())
    return t.to(device)


class Engine:
    def __init__(self, cfg: ModelConfig, store: ParamStore, max_seq: int = 4096):
        self.cfg = cfg
        self.s = store
        self.dev = store.device
        t = cfg.text
        if t.llama:
            cos, sin = rope_tables_llama3(t.head_dim, t.rope_theta, t.rope_scaling, max_seq)
        else:
            cos, sin = rope_tables(t.hidden, t.heads, t.rotary_pct, t.rope_theta, max_seq)
        self.cos = cos.to(self.dev)
        self.sin = sin.to(self.dev)
        self.cache: dict = {}
        # activation checkpointing (HF gradient_checkpointing, src/train.py:112 →
        # TrainingClass.gradient_checkpointing): keep only each layer's input residual
        # stream in the forward and recompute the layer's forward right before its
        # backward (the recompute is not counted as model FLOPs, as in the reference)
        self.checkpointing = False
        # ZeRO-3 parameter residency (zero3.Zero3Residency): gathers a unit's weights
        # before use and reduce-scatters its gradients after its backward
        self.units = None
        # weight-gradient GEMMs on a second stream (see _dw)
        # (round 1 with gemm256: slower; round 5 with the persistent gemm4p: +0.6% at the bench
        # batch, +1.4% at 32 samples per rank — profiles/r05/dw_stream/)
        self.dw_stream = os.environ.get("MMPT_DW_STREAM", "1") == "1"
        # layers of weight-gradient work the side stream may run behind the compute stream
        self.dw_depth = max(1, int(os.environ.get("MMPT_DW_DEPTH", "1")))
        # bias gradients summed by the weight-gradient GEMM itself (K.gemm_wgrad_colsum) where
        # it takes the shape; MMPT_WGRAD_COLSUM=0: a separate column-sum pass (A/B)
        self.wgrad_colsum = os.environ.get("MMPT_WGRAD_COLSUM", "1") != "0"
        self._side = None
        self._pending: list = []
        self._fences: list = []
        # gradient-ready hook: called with a flat-buffer range [lo, hi) once every
        # gradient in it is final for this micro-batch (DDP overlap, distributed.GradSync)
        self.grad_ready_hook = None
        # every weight whose input gradient is needed gets a transposed bf16 shadow
        self.head = "text.embed" if t.tie_embeddings else "text.lm_head"
        # LLaVA-pretrain freeze (src/models/llava.py:49-52): no weight gradients for the
        # tower / language model, no backward through the tower at all
        self.frozen = cfg.freeze_tower_and_llm
        store.transposed = [n for n in store.shapes if len(store.shapes[n]) == 2 and
                            n not in ("vision.patch.weight", "text.embed", "vision.pos")]
        if t.tie_embeddings:  # the tied lm_head's input gradient reads E^T
            store.transposed.append("text.embed")
        if self.frozen and not t.llama:
            raise NotImplementedError("freeze_tower_and_llm is the llava-pretrain (Llama) recipe")
        if store.device.type == "cuda":
            store.refresh_transposed()

    def reset(self) -> None:
        """Drop every per-micro-batch state after a failed forward/backward (e.g. a
        torch.cuda.OutOfMemoryError caught by find_max_mbs_pow2 / the sweep's halving
        loop): the activation cache (incl. the logits), side-stream operands and fences,
        and the ZeRO-3 residency windows, so the retry starts from a clean engine and the
        caching allocator can release the failed micro-batch's memory."""
        if self._side is not None:
            self._side.synchronize()
        self.cache.clear()
        self._pending, self._fences = [], []
        self._recomputing = False
        if self.units is not None:
            self.units.reset()

    # -------------------------------------------------------------- helpers
    _recomputing = False

    def _restore(self, key, layer_fwd, i, B, S):
        """Activation checkpointing: re-run layer i's forward from its saved input."""
        ent = self.cache.get(key)
        if ent is None or ent[0] != "ckpt":
            return
        self._recomputing = True
        try:
            layer_fwd(i, ent[1], B, S)
        finally:
            self._recomputing = False

    def _unit_fwd(self, unit: str) -> None:
        if self.units is not None:
            self.units.forward(unit)

    def _unit_bwd(self, unit: str) -> None:
        if self.units is not None:
            self.units.backward(unit)

    def _unit_done(self, unit: str) -> None:
        if self.units is not None:
            self.units.backward_done(unit)

    # fp32 units (ZeRO-2/3 with DeepSpeed's persistence threshold: the token / position
    # embeddings partitioned, zero3.Zero3Store): gathered before their forward read, their
    # gradient window opened before and reduce-scattered after their backward
    def _is_f32_unit(self, name: str) -> bool:
        return self.units is not None and name in getattr(self.s, "fp32_units", ())

    def _f32_fwd(self, name: str) -> None:
        if self._is_f32_unit(name):
            self.units.forward(name)

    def _f32_bwd(self, name: str) -> None:
        if self._is_f32_unit(name):
            self.units.backward(name)

    def _f32_done(self, name: str) -> None:
        if self._is_f32_unit(name):
            self.units.backward_done(name)

    def _grad_open(self, unit: str) -> None:
        if self.units is not None:
            self.units.open_grad(unit)

    def unit_order(self) -> list[str]:
        """Forward order of the ZeRO-3 partition units (the parameters outside the
        fp32-read region, grouped per layer / module)."""
        cfg = self.cfg
        f32 = getattr(self.s, "fp32_units", ())
        order = []
        if cfg.multimodal:
            order += ["vision.patch"] + (["vision.pos"] if "vision.pos" in f32 else [])
            order += [f"vision.layers.{i}" for i in range(cfg.vision.used_layers)]
            order += ["proj"]
        order += (["text.embed"] if "text.embed" in f32 else [])
        order += [f"text.layers.{i}" for i in range(cfg.text.layers)]
        if not cfg.text.tie_embeddings:
            order.append("text.lm_head")
        return order

    def _ready(self, prefixes):
        """Announce that the grads of every parameter whose name starts with one of
        `prefixes` are final, as maximal contiguous runs of the flat buffer."""
        if self.grad_ready_hook is None:
            return
        spans = sorted((o, o + self.s.g(n).numel()) for n, o in self.s.offsets.items()
                       if n.startswith(prefixes))
        runs: list[list[int]] = []
        for lo, hi in spans:
            if runs and lo - runs[-1][1] < 64:  # only alignment padding in between
                runs[-1][1] = hi
            else:
                runs.append([lo, hi])
        side = self._side_stream()
        if side is None:
            for lo, hi in runs:
                self.grad_ready_hook(lo, hi)
            return
        # the collective must follow this group's weight grads (side stream) and its
        # LayerNorm / bias grads (compute stream): issue it from the side stream after
        # that stream has caught up with the compute stream
        side.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(side):
            for lo, hi in runs:
                self.grad_ready_hook(lo, hi)

    def _e(self, *shape, dtype=BF16):
        return torch.empty(*shape, dtype=dtype, device=self.dev)

    def _wn(self, name):
        """parameter name of a Linear's weight (the lm_head / tied embedding have no suffix)"""
        return name if name in self.s.shapes else name + ".weight"

    def _gw(self, name):
        """gradient tensor of a weight, or None when it is frozen (freeze_tower_and_llm)"""
        wn = self._wn(name)
        return self.s.g(wn) if self.cfg.trainable(wn) else None

    def _linear(self, x, name, out=None, bias=True, epi=K.EPI_BF16, aux=None, out2=None):
        W = self.s.w(self._wn(name))
        if out is None:
            out = self._e(x.shape[0], W.shape[0], dtype=F32 if epi == K.EPI_F32_RESID else BF16)
        b = self.s.w(name + ".bias") if bias else None
        K.gemm(x, W, out, epilogue=epi, bias=b, aux=aux, out2=out2)
        return out

    def _dx(self, dy, name):
        Wt = self.s.wt(self._wn(name))
        out = self._e(dy.shape[0], Wt.shape[0])
        K.gemm(dy, Wt, out)  # dX = dY·W = dY·(W^T)^T, both operands K-contiguous
        return out

    def _dx_dgelu(self, dy, name, pre, bias_of=None, quick=False):
        """dpre = bf16(dY·W) * gelu'(pre) (quick: CLIP's quick-GELU); with bias_of, that
        layer's bias gradient Σ_rows dpre is produced by the same GEMM (column sums in the
        epilogue)."""
        Wt = self.s.wt(name + ".weight")
        out = self._e(dy.shape[0], Wt.shape[0])
        if bias_of is None:
            K.gemm(dy, Wt, out, epilogue=K.EPI_BF16_DQGELU if quick else K.EPI_BF16_DGELU,
                   aux=pre)
        else:
            K.gemm_dgelu_colsum(dy, Wt, out, pre, self.s.g(bias_of + ".bias"), quick=quick)
        return out

    def _dw(self, dy, x, name, bias=True, bias2=None):
        """Weight (and bias) gradient.  With the weight-gradient stream enabled the GEMM
        runs there, concurrently with the input-gradient chain on the compute stream
        (it fills the CUs left idle by the other kernels' last tile waves); every gradient
        element is still written by exactly one stream, in micro-batch order."""
        if not self.cfg.trainable(self._wn(name)):
            return  # frozen: no weight (or bias) gradient
        G = self.s.g(self._wn(name))
        side = self._side_stream()
        if side is None:
            self._wgrad(dy, x, G, name, bias, bias2)
            return
        side.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(side):
            self._wgrad(dy, x, G, name, bias, bias2)
        # keep the operands alive until the compute stream is ordered after this GEMM
        # (_side_fence): freeing them earlier would let the caching allocator hand their
        # memory to a compute-stream kernel while the side stream still reads it.
        # (record_stream would instead defer every reuse to GPU progress, and with the
        # host far ahead of the GPU the allocator would grow until it thrashes.)
        self._pending.extend((dy, x))

    def _wgrad(self, dy, x, G, name, bias, bias2):
        """G += dyᵀ·x and, with `bias`, name.bias (and bias2.bias) += bf16(Σ_rows dy): one
        GEMM pass when the fused form takes the shape, else the GEMM then a column sum."""
        if bias:
            db = self.s.g(name + ".bias")
            db2 = None if bias2 is None else self.s.g(bias2 + ".bias")
            if self.wgrad_colsum and K.gemm_wgrad_colsum(dy, x, G, db, db2):
                return
        K.gemm(dy, x, G, layout_a=K.K_ROWS, layout_b=K.K_ROWS, epilogue=K.EPI_F32_ACC)
        if bias:
            K.colsum(dy, db, accumulate=True, dbias2=db2)

    def _side_stream(self):
        """The weight-gradient stream (None: everything on the compute stream).  A residency
        hook may veto it (`grads_on_compute_stream`); ZeRO-2/3 (zero3.Zero3Sync) takes it since
        round 5 — its per-unit reduce waits for this stream."""
        if (not self.dw_stream or self.dev.type != "cuda" or
                getattr(self.units, "grads_on_compute_stream", False)):
            return None
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.dev)
        # ZeRO-2/3: its gradient hooks wait for this stream — handed over on every call, so a
        # residency object installed after the stream was created gets it too
        if getattr(self.units, "side", 0) is None:
            self.units.side = self._side
        return self._side

    def _side_fence(self) -> None:
        """Called as each layer's backward starts: the compute stream waits for the side
        stream's work of two layers up, then that work's operands are released — one
        layer of weight-gradient GEMMs stays in flight beside the input-gradient chain."""
        if self._side is None:
            return
        ev = torch.cuda.Event()
        ev.record(self._side)
        self._fences.append((ev, self._pending))
        self._pending = []
        while len(self._fences) > self.dw_depth:
            ev0, _ = self._fences.pop(0)
            torch.cuda.current_stream(self.dev).wait_event(ev0)

    def _join_side(self) -> None:
        if self._side is not None:
            torch.cuda.current_stream(self.dev).wait_stream(self._side)
            self._fences, self._pending = [], []

    # -------------------------------------------------------------- text layers
    def _text_layer_fwd(self, i, x, B, S):
        t = self.cfg.text
        T, h, H, D = B * S, t.hidden, t.heads, t.head_dim
        p = f"text.layers.{i}."
        y1, y2 = self._e(T, h), self._e(T, h)
        mean, rstd = self._e(T, dtype=F32), self._e(T, dtype=F32)
        K.layernorm_fwd(x, self.s.p(p + "ln1.weight"), self.s.p(p + "ln1.bias"), t.eps, y1, mean,
                        rstd, self.s.p(p + "ln2.weight"), self.s.p(p + "ln2.bias"), y2)
        qkv = self._linear(y1, p + "qkv")
        if t.rot_dims > 0:
            K.rope_inplace(qkv, S, H, D, t.rot_dims, 3 * D, D, self.cos, self.sin)
        a = self._e(T, h)
        lse = self._e(B * H * S, dtype=F32)
        K.attention_fwd(qkv, B, S, H, D, 3 * D, D, True, D ** -0.5, a, lse)
        ap = self._linear(a, p + "dense")
        pre, act = self._e(T, t.ffn), self._e(T, t.ffn)
        self._linear(y2, p + "fc1", out=pre, epi=K.EPI_BF16_GELU, out2=act)
        xn = self._e(T, h, dtype=F32)
        # h' = (mlp + attn) [bf16 add] + h [fp32]   (tf:modeling_gpt_neox.py:271-274)
        self._linear(act, p + "fc2", out=xn, epi=K.EPI_F32_RESID, aux=ap, out2=x)
        if self.checkpointing and not self._recomputing:
            self.cache[("t", i)] = ("ckpt", x)
        else:
            self.cache[("t", i)] = (x, mean, rstd, y1, y2, qkv, a, lse, pre, act)
        return xn

    def _resid_grad_targets(self, i):
        """bf16 copy + bias-gradient targets for text layer i's residual-stream gradient:
        d(fc2.bias) == d(dense.bias) == Σ bf16(dh) under the parallel residual."""
        if i < 0:
            return {}
        p = f"text.layers.{i}."
        self._grad_open(f"text.layers.{i}")
        T = self._T
        return dict(dx_bf16=self._e(T, self.cfg.text.hidden), dsum=self.s.g(p + "fc2.bias"),
                    dsum2=self.s.g(p + "dense.bias"))

    def _text_layer_bwd(self, i, dxn, ds, B, S):
        """dxn: fp32 gradient of layer i's output; ds = bf16(dxn), the grad of the bf16
        (mlp + attn) sum, produced (with the fc2/dense bias gradients) by the layer
        above's fused LayerNorm backward."""
        t = self.cfg.text
        T, h, H, D = B * S, t.hidden, t.heads, t.head_dim
        p = f"text.layers.{i}."
        self._side_fence()
        self._unit_bwd(f"text.layers.{i}")
        self._restore(("t", i), self._text_layer_fwd, i, B, S)
        x, mean, rstd, y1, y2, qkv, a, lse, pre, act = self.cache.pop(("t", i))
        dpre = self._dx_dgelu(ds, p + "fc2", pre, bias_of=p + "fc1")
        self._dw(ds, act, p + "fc2", bias=False)
        dy2 = self._dx(dpre, p + "fc1")
        self._dw(dpre, y2, p + "fc1", bias=False)
        da = self._dx(ds, p + "dense")
        self._dw(ds, a, p + "dense", bias=False)
        dqkv = self._e(T, 3 * h)
        if t.rot_dims > 0:  # + the rope backward (in the dK / dQ epilogues at D = 256)
            K.attention_bwd_rope(qkv, B, S, H, D, 3 * D, D, True, D ** -0.5, a, da, lse, dqkv,
                                 t.rot_dims, self.cos, self.sin)
        else:
            K.attention_bwd(qkv, B, S, H, D, 3 * D, D, True, D ** -0.5, a, da, lse, dqkv)
        dy1 = self._dx(dqkv, p + "qkv")
        self._dw(dqkv, y1, p + "qkv")
        # dx = dxn + LN1'(dy1) + LN2'(dy2)  (in place over dxn), + bf16 copy for layer i-1
        nxt = self._resid_grad_targets(i - 1)
        K.layernorm_bwd(x, mean, rstd, dy1, self.s.p(p + "ln1.weight"), dxn,
                        self.s.g(p + "ln1.weight"), self.s.g(p + "ln1.bias"), dy2,
                        self.s.p(p + "ln2.weight"), self.s.g(p + "ln2.weight"),
                        self.s.g(p + "ln2.bias"), dresid=dxn, **nxt)
        self._unit_done(f"text.layers.{i}")
        return dxn, nxt.get("dx_bf16")

    # -------------------------------------------------------------- llama layers
    def _llama_layer_fwd(self, i, x, B, S):
        """LlamaDecoderLayer (tf:models/llama/modeling_llama.py:284-324) under autocast:
        h = x + bf16(o_proj(attn(RMS1 x)));  x' = h + bf16(down(bf16(silu(g)) * u)), with
        g|u = gate_up(RMS2 h) in one GEMM (blocked weight, SwiGLU epilogue), q/k/v in one
        GEMM, llama3 RoPE in place, GQA flash attention."""
        t = self.cfg.text
        T, h, H, Hk, D = B * S, t.hidden, t.heads, t.n_kv, t.head_dim
        p = f"text.layers.{i}."
        y1, r1 = self._e(T, h), self._e(T, dtype=F32)
        K.rmsnorm_fwd(x, self.s.p(p + "ln1.weight"), t.eps, y1, r1)
        qkv = self._linear(y1, p + "qkv", bias=False)
        K.rope_inplace(qkv, S, H, D, D, D, 0, self.cos, self.sin, parts=1)
        K.rope_inplace(qkv, S, Hk, D, D, D, 0, self.cos, self.sin, parts=1, offset=H * D)
        a = self._e(T, h)
        lse = self._e(B * H * S, dtype=F32)
        K.attention_gqa_fwd(qkv, B, S, H, Hk, D, H * D, (H + Hk) * D, True, D ** -0.5, a, lse)
        h1 = self._linear(a, p + "dense", bias=False, epi=K.EPI_F32_RESID, out2=x)
        y2, r2 = self._e(T, h), self._e(T, dtype=F32)
        K.rmsnorm_fwd(h1, self.s.p(p + "ln2.weight"), t.eps, y2, r2)
        gu, act = self._e(T, 2 * t.ffn), self._e(T, t.ffn)
        self._linear(y2, p + "gate_up", out=gu, bias=False, epi=K.EPI_BF16_SWIGLU, out2=act)
        xn = self._linear(act, p + "down", bias=False, epi=K.EPI_F32_RESID, out2=h1)
        if self.checkpointing and not self._recomputing:
            self.cache[("t", i)] = ("ckpt", x)
        else:
            self.cache[("t", i)] = (x, r1, y1, qkv, a, lse, h1, r2, y2, gu, act)
        return xn

    def _llama_layer_bwd(self, i, dxn, ds, B, S):
        """dxn: fp32 gradient of layer i's output, ds = bf16(dxn) (the down_proj output's
        gradient).  Returns (dx, bf16(dx)) for layer i-1."""
        t = self.cfg.text
        T, h, H, Hk, D = B * S, t.hidden, t.heads, t.n_kv, t.head_dim
        p = f"text.layers.{i}."
        self._side_fence()
        self._unit_bwd(f"text.layers.{i}")
        self._restore(("t", i), self._llama_layer_fwd, i, B, S)
        x, r1, y1, qkv, a, lse, h1, r2, y2, gu, act = self.cache.pop(("t", i))
        # d act = ds·W_down -> (d gate, d up) by the SwiGLU-backward epilogue
        dgu = self._e(T, 2 * t.ffn)
        K.gemm(ds, self.s.wt(p + "down.weight"), dgu, epilogue=K.EPI_BF16_DSWIGLU, aux=gu)
        self._dw(ds, act, p + "down", bias=False)
        dy2 = self._dx(dgu, p + "gate_up")
        self._dw(dgu, y2, p + "gate_up", bias=False)
        # dh1 = dxn + RMS2'(dy2) (in place); d1 = bf16(dh1), the o_proj output's gradient
        d1 = self._e(T, h)
        K.rmsnorm_bwd(h1, r2, dy2, self.s.p(p + "ln2.weight"), dxn, dw=self._gw(p + "ln2"),
                      dresid=dxn, dx_bf16=d1)
        da = self._dx(d1, p + "dense")
        self._dw(d1, a, p + "dense", bias=False)
        dqkv = self._e(T, t.qkv_dim)
        K.attention_gqa_bwd(qkv, B, S, H, Hk, D, H * D, (H + Hk) * D, True, D ** -0.5, a, da, lse,
                            dqkv)
        K.rope_inplace(dqkv, S, H, D, D, D, 0, self.cos, self.sin, inverse=True, parts=1)
        K.rope_inplace(dqkv, S, Hk, D, D, D, 0, self.cos, self.sin, inverse=True, parts=1,
                       offset=H * D)
        dy1 = self._dx(dqkv, p + "qkv")
        self._dw(dqkv, y1, p + "qkv", bias=False)
        nxt = self._e(T, h) if i > 0 else None
        K.rmsnorm_bwd(x, r1, dy1, self.s.p(p + "ln1.weight"), dxn, dw=self._gw(p + "ln1"),
                      dresid=dxn, dx_bf16=nxt)
        self._unit_done(f"text.layers.{i}")
        return dxn, nxt

    # -------------------------------------------------------------- vision
    def _vit_layer_fwd(self, i, x, B, Sv):
        v = self.cfg.vision
        T, h, H, D = B * Sv, v.hidden, v.heads, v.head_dim
        p = f"vision.layers.{i}."
        y1 = self._e(T, h)
        m1, r1 = self._e(T, dtype=F32), self._e(T, dtype=F32)
        K.layernorm_fwd(x, self.s.p(p + "ln1.weight"), self.s.p(p + "ln1.bias"), v.eps, y1, m1, r1)
        qkv = self._linear(y1, p + "qkv")
        a = self._e(T, h)
        lse = self._e(B * H * Sv, dtype=F32)
        K.attention_fwd(qkv, B, Sv, H, D, D, h, False, D ** -0.5, a, lse)
        h1 = self._linear(a, p + "o", epi=K.EPI_F32_RESID, out2=x)
        y2 = self._e(T, h)
        m2, r2 = self._e(T, dtype=F32), self._e(T, dtype=F32)
        K.layernorm_fwd(h1, self.s.p(p + "ln2.weight"), self.s.p(p + "ln2.bias"), v.eps, y2, m2, r2)
        pre, act = self._e(T, v.ffn), self._e(T, v.ffn)
        self._linear(y2, p + "fc1", out=pre, out2=act,
                     epi=K.EPI_BF16_QGELU if v.act == "quick_gelu" else K.EPI_BF16_GELU)
        xn = self._linear(act, p + "fc2", epi=K.EPI_F32_RESID, out2=h1)
        if self.frozen:
            pass  # frozen tower: no backward through it, nothing to keep
        elif self.checkpointing and not self._recomputing:
            self.cache[("v", i)] = ("ckpt", x)
        else:
            self.cache[("v", i)] = (x, m1, r1, y1, qkv, a, lse, h1, m2, r2, y2, pre, act)
        return xn

    def _vit_layer_bwd(self, i, dxn, d2, B, Sv):
        """d2 = bf16(dxn) with fc2.bias's gradient already accumulated (by the layer
        above's fused LN backward, or the caller for the top layer)."""
        v = self.cfg.vision
        T, h, H, D = B * Sv, v.hidden, v.heads, v.head_dim
        p = f"vision.layers.{i}."
        self._side_fence()
        self._unit_bwd(f"vision.layers.{i}")
        self._restore(("v", i), self._vit_layer_fwd, i, B, Sv)
        x, m1, r1, y1, qkv, a, lse, h1, m2, r2, y2, pre, act = self.cache.pop(("v", i))
        dpre = self._dx_dgelu(d2, p + "fc2", pre, bias_of=p + "fc1", quick=v.act == "quick_gelu")
        self._dw(d2, act, p + "fc2", bias=False)
        dy2 = self._dx(dpre, p + "fc1")
        self._dw(dpre, y2, p + "fc1", bias=False)
        # dh1 = dxn + LN2'(dy2)   (in place), d1 = bf16(dh1), d(o.bias) = Σ d1
        d1 = self._e(T, h)
        K.layernorm_bwd(h1, m2, r2, dy2, self.s.p(p + "ln2.weight"), dxn,
                        self.s.g(p + "ln2.weight"), self.s.g(p + "ln2.bias"), dresid=dxn,
                        dx_bf16=d1, dsum=self.s.g(p + "o.bias"))
        da = self._dx(d1, p + "o")
        self._dw(d1, a, p + "o", bias=False)
        dqkv = self._e(T, 3 * h)
        K.attention_bwd(qkv, B, Sv, H, D, D, h, False, D ** -0.5, a, da, lse, dqkv)
        dy1 = self._dx(dqkv, p + "qkv")
        self._dw(dqkv, y1, p + "qkv")
        if i > 0:
            self._grad_open(f"vision.layers.{i - 1}")
        nxt = {} if i == 0 else dict(dx_bf16=self._e(T, h),
                                     dsum=self.s.g(f"vision.layers.{i - 1}.fc2.bias"))
        K.layernorm_bwd(x, m1, r1, dy1, self.s.p(p + "ln1.weight"), dxn,
                        self.s.g(p + "ln1.weight"), self.s.g(p + "ln1.bias"), dresid=dxn, **nxt)
        self._unit_done(f"vision.layers.{i}")
        return dxn, nxt.get("dx_bf16")

    def _vision_fwd(self, pixels, B):
        v = self.cfg.vision
        npch, hv = v.num_patches, v.hidden
        cols = self._e(B * npch, v.patch_k)
        K.im2col(pixels, v.patch, cols)
        self._unit_fwd("vision.patch")
        po = self._linear(cols, "vision.patch", bias=v.patch_bias)
        h = self._e(B * (npch + 1), hv, dtype=F32)
        self._f32_fwd("vision.pos")
        K.vit_embed_fwd(B, npch, po, self.s.p("vision.cls"), self.s.p("vision.pos"), h)
        pre_ln = None
        if v.pre_ln:  # CLIP pre_layrnorm: fp32 in, fp32 residual stream out
            e = h
            h = self._e(B * (npch + 1), hv, dtype=F32)
            m0, r0 = self._e(B * (npch + 1), dtype=F32), self._e(B * (npch + 1), dtype=F32)
            K.layernorm_f32_fwd(e, self.s.p("vision.ln_pre.weight"), self.s.p("vision.ln_pre.bias"),
                                v.eps, h, m0, r0)
            pre_ln = (e, m0, r0)
        for i in range(v.used_layers):
            self._unit_fwd(f"vision.layers.{i}")
            h = self._vit_layer_fwd(i, h, B, npch + 1)
        f = self._e(B * npch, hv)
        K.select_patches_fwd(B, npch, h, f)
        ht = self.cfg.text.hidden
        ppre, pact = self._e(B * npch, ht), self._e(B * npch, ht)
        self._unit_fwd("proj")
        self._linear(f, "proj.fc1", out=ppre, epi=K.EPI_BF16_GELU, out2=pact)
        img = self._linear(pact, "proj.fc2")
        self.cache["vis"] = (cols, f, ppre, pact, pre_ln)
        return img

    def _vision_bwd(self, dimg, B):
        v = self.cfg.vision
        npch, hv = v.num_patches, v.hidden
        cols, f, ppre, pact, pre_ln = self.cache.pop("vis")
        self._side_fence()
        self._unit_bwd("proj")
        dppre = self._dx_dgelu(dimg, "proj.fc2", ppre, bias_of="proj.fc1")
        self._dw(dimg, pact, "proj.fc2")
        if self.frozen:  # the tower is frozen: nothing below the projector needs a gradient
            self._dw(dppre, f, "proj.fc1", bias=False)
            self._unit_done("proj")
            return
        df = self._dx(dppre, "proj.fc1")
        self._dw(dppre, f, "proj.fc1", bias=False)
        self._unit_done("proj")
        dh = self._e(B * (npch + 1), hv, dtype=F32)
        K.select_patches_bwd(B, npch, df, dh, accumulate=False)
        top = v.used_layers - 1
        self._grad_open(f"vision.layers.{top}")
        d2 = self._e(B * (npch + 1), hv)
        K.cast_f32_bf16(dh, d2)
        K.colsum(d2, self.s.g(f"vision.layers.{top}.fc2.bias"), accumulate=True)
        for i in reversed(range(v.used_layers)):
            dh, d2 = self._vit_layer_bwd(i, dh, d2, B, npch + 1)
        if pre_ln is not None:  # through pre_layrnorm (its γ/β grads accumulate)
            e, m0, r0 = pre_ln
            de = torch.empty_like(dh)
            K.layernorm_f32_bwd(e, m0, r0, dh, self.s.p("vision.ln_pre.weight"), de,
                                self.s.g("vision.ln_pre.weight"), self.s.g("vision.ln_pre.bias"))
            dh = de
        dpo = self._e(B * npch, hv)
        self._f32_bwd("vision.pos")
        K.vit_embed_bwd(B, npch, dh, self.s.g("vision.cls"), self.s.g("vision.pos"), dpo)
        self._f32_done("vision.pos")
        self._unit_bwd("vision.patch")
        self._dw(dpo, cols, "vision.patch", bias=v.patch_bias)
        self._unit_done("vision.patch")

    # -------------------------------------------------------------- whole model
    def forward(self, batch: Batch, grad_scale: float, need_grad: bool = True) -> torch.Tensor:
        """Returns Σ_tokens CE (device fp32 [1]); when need_grad, dlogits are written
        (scaled by grad_scale = 1/num_items of the global batch) and the caches kept."""
        cfg, t = self.cfg, self.cfg.text
        B, S = batch.B, batch.S
        T = B * S
        if self.dev.type == "cuda":
            batch.use(torch.cuda.current_stream(self.dev))
        region = getattr(self.units, "region", None)
        if region is not None:  # an overlapped optimizer update of the fp32-read region
            region()
        if S > self.cos.shape[0]:
            raise ValueError(f"sequence {S} longer than the rope table {self.cos.shape[0]}")
        img = self._vision_fwd(batch.pixels, B) if cfg.multimodal else None
        h = self._e(T, t.hidden, dtype=F32)
        self._f32_fwd("text.embed")
        K.embed_fwd(batch.ids, self.s.p("text.embed"), h, batch.img_map, img)
        layer_fwd = self._llama_layer_fwd if t.llama else self._text_layer_fwd
        for i in range(t.layers):
            self._unit_fwd(f"text.layers.{i}")
            h = layer_fwd(i, h, B, S)
        yf = self._e(T, t.hidden)
        mf, rf = self._e(T, dtype=F32), self._e(T, dtype=F32)
        if t.llama:
            K.rmsnorm_fwd(h, self.s.p("text.final_ln.weight"), t.eps, yf, rf)
        else:
            K.layernorm_fwd(h, self.s.p("text.final_ln.weight"), self.s.p("text.final_ln.bias"),
                            t.eps, yf, mf, rf)
        if batch.loss_rows is not None:  # compact the loss rows (image slots carry no label)
            yv = self._e(batch.loss_rows.numel(), t.hidden)
            K.gather_rows(yf, batch.loss_rows, yv)
            yf = yv
        logits = self._e(yf.shape[0], t.vocab)
        if self.head == "text.lm_head":
            self._unit_fwd("text.lm_head")
        K.gemm(yf, self.s.w(self.head), logits)
        loss_rows = self._e(yf.shape[0], dtype=F32)
        K.cross_entropy(logits, batch.loss_labels, -100, grad_scale, loss_rows,
                        logits if need_grad else None, vocab_valid=t.n_vocab)
        loss = self._e(1, dtype=F32)
        K.sum_f32(loss_rows, loss)
        if need_grad:
            self.cache["head"] = (h, mf, rf, yf, logits)
        else:
            self.cache.clear()
        return loss

    def backward(self, batch: Batch, scale: torch.Tensor | None = None) -> None:
        """Accumulates every parameter gradient into the flat grad buffer.  `scale`
        (device scalar, e.g. autograd's grad_output) multiplies the loss gradient."""
        cfg, t = self.cfg, self.cfg.text
        B, S = batch.B, batch.S
        hL, mf, rf, yf, dlogits = self.cache.pop("head")
        if scale is not None:
            dlogits.mul_(scale.to(torch.float32))
        tied = self.head == "text.embed"
        if not tied:
            self._unit_bwd("text.lm_head")
        dyf = self._dx(dlogits, self.head)
        self._dw(dlogits, yf, self.head, bias=False)
        if not tied:
            self._unit_done("text.lm_head")
        del dlogits
        if batch.loss_map is not None:  # back to every row (zero where the label is ignored)
            dyc = dyf
            dyf = self._e(hL.shape[0], t.hidden)
            K.expand_rows(dyc, batch.loss_map, dyf)
        dh = torch.empty_like(hL)
        self._T = B * S
        if t.llama:
            ds = self._e(B * S, t.hidden)
            K.rmsnorm_bwd(hL, rf, dyf, self.s.p("text.final_ln.weight"), dh,
                          dw=self._gw("text.final_ln"), dx_bf16=ds)
            layer_bwd = self._llama_layer_bwd
        else:
            top = self._resid_grad_targets(t.layers - 1)
            K.layernorm_bwd(hL, mf, rf, dyf, self.s.p("text.final_ln.weight"), dh,
                            self.s.g("text.final_ln.weight"), self.s.g("text.final_ln.bias"), **top)
            ds = top["dx_bf16"]
            layer_bwd = self._text_layer_bwd
        self._ready(("text.final_ln.",) + (() if tied else ("text.lm_head",)))
        for i in reversed(range(t.layers)):
            dh, ds = layer_bwd(i, dh, ds, B, S)
            self._ready((f"text.layers.{i}.",))
        dimg = self._e(B * cfg.vision.num_patches, t.hidden) if cfg.multimodal else None
        self._f32_bwd("text.embed")
        K.embed_bwd(batch.segments, dh, None if self.frozen else self.s.g("text.embed"),
                    batch.img_map, dimg)
        self._f32_done("text.embed")
        self._ready(("text.embed",))
        if cfg.multimodal:
            self._vision_bwd(dimg, B)
            self._ready(("vision.", "proj."))
        self._join_side()
        self.cache.clear()
