"""ZeRO-3 (DeepSpeed stage 3 / FSDP FULL_SHARD) over RCCL: parameters, gradients and
optimizer state partitioned across the data-parallel ranks, parameters gathered per
layer just before use and gradients reduce-scattered per layer right after their
backward (src/train.py:170-194 → DeepSpeed `zero_optimization.stage = 3`;
experiments/config.py:56-74 `sharding = "zero_3" | "fsdp_full_shard"`).

Layout (per rank, all in HBM):

* the **persistent region** — every parameter the step reads from the fp32 master
  (LayerNorm γ/β, token embedding, ViT CLS/position embeddings, `params.is_fp32_read`)
  stays replicated, like DeepSpeed's `stage3_param_persistence_threshold` params: its
  fp32 master / grad live in full on every rank, its grads are all-reduced once per
  optimizer step and every rank applies the identical update;
* one **unit** per layer / module (`Engine.unit_order`: ViT patch, ViT layers,
  projector, text layers, lm_head): the unit's parameters are packed into a virtual
  flat range padded to a multiple of 64·world, and this rank keeps only its 1/world
  slice of the fp32 master, fp32 grad, Adam m/v and bf16 shadow;
* **windows**: two bf16 gather windows (the unit in use + the prefetched next unit),
  one transposed-weight window (rebuilt from the gathered weights by the transpose
  kernel for the input-gradient GEMMs) and two fp32 gradient windows (the unit being
  back-propagated + the layer below, whose residual bias grads the fused LayerNorm
  backward produces one layer early).

Streams: gathers and reduce-scatters run on a dedicated communication stream, ordered
against the compute stream with events only (no host sync): the gather of unit k+1 is
issued when unit k starts, so it overlaps unit k's GEMMs; the reduce-scatter of unit k's
gradients overlaps unit k-1's backward.
"""

from __future__ import annotations

import math
import os

import torch
import torch.distributed as dist

from .distributed import COMM_TIMER, _Comm, force_collectives
from .params import ALIGN, _round, is_fp32_read


def unit_of(name: str) -> str | None:
    """Partition unit of a parameter (None = persistent, replicated)."""
    if is_fp32_read(name):
        return None
    if name.startswith(("text.layers.", "vision.layers.")):
        return ".".join(name.split(".")[:3])
    if name.startswith("proj."):
        return "proj"
    if name.startswith("vision.patch."):
        return "vision.patch"
    if name == "text.lm_head":
        return "text.lm_head"
    raise KeyError(f"no ZeRO-3 unit for parameter {name!r}")


class _Unit:
    __slots__ = ("name", "offsets", "size", "shard", "local_lo", "rep_lo")

    def __init__(self, name):
        self.name, self.offsets, self.size, self.shard, self.local_lo = name, {}, 0, 0, 0
        self.rep_lo = 0  # replicate mode: the unit's offset in the full bf16 copy


class Zero3Store:
    """ParamStore-compatible accessors (p / w / wt / g) over the ZeRO-3 partition.
    `w`, `wt` and a unit parameter's `g` resolve to the window the unit is bound to
    (Zero3Sync binds them); touching an unbound unit raises.

    replicate=True is ZeRO-2 (DeepSpeed stage 2, FSDP SHARD_GRAD_OP, src/train.py:170-181):
    the same partition of the fp32 master, gradients and Adam state, the same per-unit
    gradient windows reduce-scattered into the shard after each unit's backward — but the
    bf16 weights stay replicated: one full bf16 copy (`rep_w`) and its transposes
    (`rep_wt`) on every rank, refreshed once per optimizer step by a per-unit all-gather of
    the updated shards (Zero3Sync, lazily before each unit's first use).  No full fp32
    master or gradient buffer exists on any rank.

    persist_threshold (DeepSpeed `stage3_param_persistence_threshold`, "auto" = 10 x hidden,
    src/train.py:182-194 via tf:integrations/deepspeed.py): a parameter the step reads as
    fp32 (`params.is_fp32_read`) stays replicated only at or below it — LayerNorm gamma/beta, the
    ViT CLS token (DeepSpeed keeps ds_numel <= threshold persistent).  Above it (the token
    embedding: 103 M elements for Pythia-1B; the ViT position embedding) it becomes an **fp32 unit**: partitioned like every other unit (fp32
    master, gradient and Adam state 1/world per rank), all-gathered in fp32 before its
    forward use (ZeRO-3: into an fp32 window; ZeRO-2: into a replicated fp32 copy refreshed
    once per step) and its gradient reduce-scattered after its backward.  The fp32 units are
    laid out right after the persistent region, so [0, fp32_keep) is the part of the local
    master an optimizer offload keeps (and uploads) in fp32.  None = every fp32-read
    parameter persistent (the round-3 layout; also the tied-embedding case, whose bf16
    transpose the lm_head reads)."""

    def __init__(self, shapes: dict[str, tuple[int, ...]], device: torch.device | str,
                 world: int = 1, rank: int = 0, replicate: bool = False,
                 persist_threshold: int | None = None):
        self.shapes = dict(shapes)
        self.device = torch.device(device)
        self.world, self.rank = world, rank
        self.persist_threshold = persist_threshold
        self.fp32_units = [n for n in self.shapes if is_fp32_read(n) and persist_threshold is not None
                           and math.prod(self.shapes[n]) > persist_threshold]
        self.offsets: dict[str, int] = {}  # persistent params: local offset
        off = 0
        for n in self.shapes:
            if is_fp32_read(n) and n not in self.fp32_units:
                self.offsets[n] = off
                off += _round(math.prod(self.shapes[n]), ALIGN)
        self.fp32_end = off
        self.units: dict[str, _Unit] = {}
        for n in self.fp32_units + [n for n in self.shapes if n not in self.fp32_units]:
            u = self.unit_of(n)
            if u is None:
                continue
            unit = self.units.setdefault(u, _Unit(u))
            unit.offsets[n] = unit.size
            unit.size += _round(math.prod(self.shapes[n]), ALIGN)
        for unit in self.units.values():
            unit.size = _round(unit.size, ALIGN * world)
            unit.shard = unit.size // world
            unit.local_lo = off
            off += unit.shard
        # [0, fp32_keep): the persistent region + the fp32 units' shards (read as fp32)
        self.fp32_keep = self.fp32_end + sum(self.units[u].shard for u in self.fp32_units)
        self.numel = off  # local elements
        self.shard_size = off
        self.padded = off
        self.max_unit = max(u.size for u in self.units.values())
        self.replicate = replicate
        f32, bf = torch.float32, torch.bfloat16
        self.master = torch.zeros(off, dtype=f32, device=self.device)
        self.shadow = torch.zeros(off, dtype=bf, device=self.device)
        self.grad = torch.zeros(off, dtype=f32, device=self.device)
        bf_max = max([u.size for n, u in self.units.items() if n not in self.fp32_units] or [64])
        f32_max = max([self.units[u].size for u in self.fp32_units] or [0])
        if replicate:
            rep = rep32 = 0
            for n, unit in self.units.items():
                if n in self.fp32_units:
                    unit.rep_lo, rep32 = rep32, rep32 + unit.size
                else:
                    unit.rep_lo, rep = rep, rep + unit.size
            self.rep_w = torch.zeros(rep, dtype=bf, device=self.device)
            self.rep_wt = torch.zeros(rep, dtype=bf, device=self.device)
            self.rep_f32 = torch.zeros(rep32, dtype=f32, device=self.device)
            self.win_w, self.win_wt, self.win_f32 = [], None, None
        else:
            self.win_w = [torch.zeros(bf_max, dtype=bf, device=self.device) for _ in range(2)]
            self.win_wt = torch.zeros(bf_max, dtype=bf, device=self.device)
            self.win_f32 = torch.zeros(f32_max, dtype=f32, device=self.device) if f32_max else None
        self.bound_f32: str | None = None  # the fp32 unit the fp32 window holds (ZeRO-3)
        self.win_g = [torch.zeros(self.max_unit, dtype=f32, device=self.device) for _ in range(2)]
        # transposed bf16 copies of replicated (persistent) weights the step multiplies by:
        # the tied lm_head's embedding (Llama), built by refresh_transposed
        self.pers_wt: dict[str, torch.Tensor] = {}
        self.bound_w: dict[str, int] = {}
        self.alias_w = False  # set by Zero3Sync.direct: w() reads the shard in place
        self.bound_wt: str | None = None
        self.bound_g: dict[str, int] = {}
        self.transposed: list[str] = []

    # ------------------------------------------------------------ accessors
    def names(self):
        return list(self.shapes)

    def unit_of(self, name: str) -> str | None:
        """Partition unit of a parameter in this layout (fp32 units are named after their
        parameter; None = persistent)."""
        return name if name in self.fp32_units else unit_of(name)

    def _loc(self, name):
        u = self.unit_of(name)
        return u, self.units[u].offsets[name] if u is not None else self.offsets[name]

    def p(self, name: str) -> torch.Tensor:
        u, o = self._loc(name)
        n = math.prod(self.shapes[name])
        if u is not None and u in self.fp32_units:  # the gathered fp32 values
            if self.replicate:
                lo = self.units[u].rep_lo + o
                return self.rep_f32[lo:lo + n].view(self.shapes[name])
            if self.bound_f32 != u:
                raise RuntimeError(f"ZeRO-3: fp32 unit {u} used before it was gathered")
            return self.win_f32[o:o + n].view(self.shapes[name])
        if u is not None:
            raise RuntimeError(f"ZeRO-3: {name} is partitioned (no full fp32 master on a rank)")
        return self.master[o:o + n].view(self.shapes[name])

    def w(self, name: str) -> torch.Tensor:
        u, o = self._loc(name)
        n = math.prod(self.shapes[name])
        if u is None:  # replicated region: its bf16 shadow is full on every rank
            return self.shadow[o:o + n].view(self.shapes[name])
        if u in self.fp32_units:
            raise RuntimeError(f"ZeRO: {name} is read in fp32 (no bf16 copy)")
        if self.replicate:
            lo = self.units[u].rep_lo + o
            return self.rep_w[lo:lo + n].view(self.shapes[name])
        slot = self.bound_w.get(u)
        if slot is None:
            raise RuntimeError(f"ZeRO-3: unit {u} used before it was gathered")
        if self.alias_w:  # world 1, no collectives: the unit's shard IS the gathered unit
            lo = self.units[u].local_lo + o
            return self.shadow[lo:lo + n].view(self.shapes[name])
        return self.win_w[slot][o:o + n].view(self.shapes[name])

    def wt(self, name: str) -> torch.Tensor:
        u, o = self._loc(name)
        r, c = self.shapes[name]
        if u is None:
            t = self.pers_wt.get(name)
            if t is None:
                raise RuntimeError(f"ZeRO: transposed copy of {name} not built")
            return t
        if self.replicate:
            lo = self.units[u].rep_lo + o
            return self.rep_wt[lo:lo + r * c].view(c, r)
        if self.bound_wt != u:
            raise RuntimeError(f"ZeRO-3: transposed weights of unit {u} not built")
        return self.win_wt[o:o + r * c].view(c, r)

    def g(self, name: str) -> torch.Tensor:
        u, o = self._loc(name)
        n = math.prod(self.shapes[name])
        if u is None:
            return self.grad[o:o + n].view(self.shapes[name])
        slot = self.bound_g.get(u)
        if slot is None:
            raise RuntimeError(f"ZeRO-3: gradient window of unit {u} not open")
        if slot < 0:  # world 1, no collectives: the unit's shard IS the unit (Zero3Sync.direct)
            lo = self.units[u].local_lo + o
            return self.grad[lo:lo + n].view(self.shapes[name])
        return self.win_g[slot][o:o + n].view(self.shapes[name])

    def local_shard(self, buf: torch.Tensor, unit: str) -> torch.Tensor:
        u = self.units[unit]
        return buf[u.local_lo:u.local_lo + u.shard]

    # ---- optimizer offload: the unit shards' fp32 master lives on the host (same local
    # layout), the device keeps the replicated region the step reads as fp32
    host_master: torch.Tensor | None = None

    def release_master(self, keep: int, host: torch.Tensor, host_lo: int = 0) -> torch.Tensor:
        self.master = self.master[:keep].clone()
        self.host_master = host
        return self.master

    def restore_master(self) -> torch.Tensor:
        if self.host_master is None:
            return self.master
        full = self.host_master.to(self.device, copy=True)
        full[:self.master.numel()].copy_(self.master)
        self.master, self.host_master = full, None
        return full

    # ------------------------------------------------------------ state
    def load(self, tensors: dict[str, torch.Tensor]) -> None:
        """Scatter full tensors into this rank's partition (replicate mode: the full bf16
        copy too, rounded like the cast kernel: round to nearest even)."""
        for name, t in tensors.items():
            flat = t.detach().reshape(-1).to(self.device, torch.float32)
            u, o = self._loc(name)
            if u is None:
                self.master[o:o + flat.numel()].copy_(flat)
                if self.host_master is not None:
                    self.host_master[o:o + flat.numel()].copy_(flat.cpu())
                continue
            unit = self.units[u]
            if self.replicate:
                lo = unit.rep_lo + o
                if u in self.fp32_units:
                    self.rep_f32[lo:lo + flat.numel()].copy_(flat)
                else:
                    self.rep_w[lo:lo + flat.numel()].copy_(flat.to(torch.bfloat16))
            s0 = self.rank * unit.shard
            lo, hi = max(o, s0), min(o + flat.numel(), s0 + unit.shard)
            if lo < hi:
                dst = unit.local_lo + lo - s0
                if self.host_master is not None:  # offload: the host master (same layout)
                    self.host_master[dst:dst + hi - lo].copy_(flat[lo - o:hi - o].cpu())
                else:
                    self.master[dst:dst + hi - lo].copy_(flat[lo - o:hi - o])
        # replicate mode: the full bf16 copy changed, so its transposes are stale — rebuild
        # them now (a Zero3Sync only re-transposes units IT marked stale after a step)
        if self.replicate and self.transposed:
            loaded = set(tensors)
            self.refresh_transposed([n for n in self.transposed
                                     if n in loaded and self.unit_of(n) is not None])

    def full_master(self, group=None) -> dict[str, torch.Tensor]:
        """All-gather the fp32 master into full tensors (collective: every rank calls)."""
        out = {n: self.p(n).detach().clone() for n in self.offsets}
        src = self.master if self.host_master is None else self.host_master
        for u, unit in self.units.items():
            full = torch.empty(unit.size, dtype=torch.float32, device=self.device)
            _all_gather(full, self.local_shard(src, u).to(self.device), group, self.world)
            for n, o in unit.offsets.items():
                out[n] = full[o:o + math.prod(self.shapes[n])].view(self.shapes[n]).clone()
        return out

    def state_dict(self) -> dict[str, torch.Tensor]:
        return self.full_master()

    def refresh_shadow(self) -> None:
        from . import kernels as K

        K.cast_f32_bf16(self.master, self.shadow[:self.master.numel()])
        if self.host_master is not None:  # released master: the unit shards from the host
            keep = self.master.numel()
            self.shadow[keep:].copy_(self.host_master[keep:].to(torch.bfloat16))
        # the transposed copies read the bf16 weights just written (replicate mode: every
        # unit's rep_wt; both modes: the persistent tied embedding's pers_wt)
        self.refresh_transposed()

    def refresh_transposed(self, names=None) -> None:
        """Transposed copies of the replicated weights the step reads transposed (the tied
        lm_head's embedding), and in replicate mode of every unit weight; ZeRO-3 rebuilds
        a unit's transposes per use inside the backward (Zero3Sync)."""
        from . import kernels as K

        for n in self.transposed if names is None else names:
            u, _ = self._loc(n)
            if u is None:
                r, c = self.shapes[n]
                if n not in self.pers_wt:
                    self.pers_wt[n] = torch.empty(c, r, dtype=torch.bfloat16, device=self.device)
                K.transpose_bf16(self.w(n), self.pers_wt[n])
            elif self.replicate:
                K.transpose_bf16(self.w(n), self.wt(n))

    def refresh_unit_transposed(self, unit: str) -> None:
        """replicate mode: rebuild one unit's transposes after its all-gather landed."""
        from . import kernels as K

        for n in self.units[unit].offsets:
            if n in self.transposed:
                K.transpose_bf16(self.w(n), self.wt(n))

    def zero_grad(self) -> None:
        self.grad.zero_()


def _all_gather(out, inp, group, world):
    if world == 1 and not force_collectives():
        out.copy_(inp)
    else:
        dist.all_gather_into_tensor(out, inp, group=group)


def _all_to_all(out, inp, group, world):
    """Equal-split all-to-all of flat buffers: out's chunk r = rank r's chunk `rank` of inp."""
    if world == 1 and not force_collectives():
        out.copy_(inp)
    elif out.is_cuda and dist.get_backend(group) == "gloo":
        # gloo has no CUDA all-to-all: gather every rank's send buffer and keep our chunks
        # (test configurations only — the GPU runs use RCCL)
        rank = dist.get_rank(group)
        c = inp.numel() // world
        allbuf = torch.empty(world * inp.numel(), dtype=inp.dtype, device=inp.device)
        dist.all_gather_into_tensor(allbuf, inp, group=group)
        out.view(world, c).copy_(allbuf.view(world, world, c)[:, rank])
    else:
        dist.all_to_all_single(out, inp, group=group)


class Zero3Sync:
    """Residency manager (the engine's `units` hook) + the step-level exchange
    (GradSync interface: reduce_grads / all_reduce_scalar / gather_params)."""

    mode = "zero3"
    # (round 5) the weight-gradient stream is allowed: windows are still opened / zeroed on
    # the compute stream, which the side stream waits for before each weight-gradient GEMM
    # (Engine._dw), and a unit's reduce / final hooks wait for the side stream (`side`,
    # set by Engine._side_stream; _comm_after_grads)
    grads_on_compute_stream = False
    side = None

    def __init__(self, store: Zero3Store, order: list[str], group=None, quant: bool = False):
        """quant: ZeRO++ (`sharding = "zero_3++"`, src/train.py:196-201) — int8 blockwise
        weight all-gather (qwZ) and int4 gradient all-to-all reduce-scatter (qgZ); the fp32
        master, Adam state and the persistent region stay exact.

        A replicate-mode store (ZeRO-2) keeps every unit's bf16 weights resident: a unit is
        all-gathered into the full copy once per optimizer step, lazily before its first use
        (prefetching the next stale unit on the comm stream, gated by the offload host
        update like a ZeRO-3 gather), and its transposes rebuilt; the gradient path is
        ZeRO-3's (windows, per-unit reduce-scatter into the shard, every micro-batch)."""
        self.s, self.group = store, group
        self.replicate = getattr(store, "replicate", False)
        if self.replicate:
            self.mode = "zero2"
            self.stale: set[str] = set()
            self.rep_ready: dict[str, object] = {}
        self.world = store.world
        self.quant = quant
        self.active = self.world > 1 or force_collectives()  # run the collectives
        # world 1 without collectives (round 5): the backward accumulates straight into the
        # gradient shard — no window zeroing, no window -> shard copy and add per unit and
        # micro-batch (1.7 ms each at C5's unit size; 400 ms of the C5 step on one GPU)
        # (MMPT_ZERO_WINDOWS=1: the window path at world 1 too, for A/B)
        self.direct = not self.active and os.environ.get("MMPT_ZERO_WINDOWS") != "1"
        # ... and the forward / backward read each unit's bf16 shard in place instead of a
        # gathered copy (the world-1 "gather" was a device copy per unit and pass)
        store.alias_w = self.direct and not self.replicate
        # fp32 units (Zero3Store persist_threshold) live outside the bf16 window rotation:
        # gathered in fp32, prefetched when the unit before them in forward order is acquired
        self.f32 = set(getattr(store, "fp32_units", ()))
        self.f32_next = {order[i - 1]: u for i, u in enumerate(order) if u in self.f32 and i > 0}
        self.f32_ready: dict[str, object] = {}  # fp32 unit -> event of its issued gather
        order = [u for u in order if u not in self.f32]
        self.fwd_order = list(order)
        self.bwd_order = list(reversed(order))
        self.cuda = store.device.type == "cuda"
        self.stream = torch.cuda.Stream(device=store.device) if self.cuda else None
        self.res: list[str | None] = [None, None]  # unit held by each gather window
        self.w_ready: list = [None, None]
        self.cur: int | None = None
        self.rs_done: list = [None, None]
        self.rs_seq = [-1, -1]  # when each gradient window was last handed to the comm stream
        self.rs_tmp = [torch.empty(max(u.shard for u in store.units.values()),
                                   dtype=torch.float32, device=store.device) for _ in range(2)]
        self.stats = {"gathers": 0, "reduce_scatters": 0}
        # overlapped offload (offload.HostAdam): `param_gate(unit, stream)` makes the comm
        # stream wait for the host update of the unit's shard before it is gathered;
        # `grad_final_hook(lo, hi, stream)` is told when a unit's gradient shard is final
        # (reduce-scatter of the step's last micro-batch, `final_pass`)
        self.param_gate = None
        self.grad_final_hook = None
        self.final_pass = False
        if quant and self.active:
            from . import kernels as K

            dev, w = store.device, self.world
            sh = max(u.shard for u in store.units.values())
            nb = K.quant_blocks(sh)
            self.q8_local = torch.empty(sh, dtype=torch.int8, device=dev)
            self.qs_local = torch.empty(nb, dtype=torch.float32, device=dev)
            self.q8_all = torch.empty(w * sh, dtype=torch.int8, device=dev)
            self.qs_all = torch.empty(w * nb, dtype=torch.float32, device=dev)
            self.q4_send = torch.empty(w * sh // 2, dtype=torch.uint8, device=dev)
            self.q4_recv = torch.empty(w * sh // 2, dtype=torch.uint8, device=dev)
            self.q4s_send = torch.empty(w * nb, dtype=torch.float32, device=dev)
            self.q4s_recv = torch.empty(w * nb, dtype=torch.float32, device=dev)

    # ------------------------------------------------------------ stream helpers
    def _compute(self):
        return torch.cuda.current_stream(self.s.device)

    def _comm_after_compute(self):
        if self.cuda:
            self.stream.wait_stream(self._compute())

    def _comm_after_grads(self):
        """Before a unit's gradient leaves (reduce-scatter / final hook): the compute stream's
        writers and the weight-gradient stream's GEMMs issued so far are enqueued."""
        self._comm_after_compute()
        if self.cuda and self.side is not None:
            self.stream.wait_stream(self.side)

    def _on_comm(self):
        return _Comm(self.stream) if self.cuda else _Null()

    def _event(self):
        if not self.cuda:
            return None
        ev = torch.cuda.Event()
        ev.record(self.stream)
        return ev

    def _wait(self, ev):
        if self.cuda and ev is not None:
            cur = self._compute()
            COMM_TIMER.wait(cur, lambda: cur.wait_event(ev))

    # ------------------------------------------------------------ gathers
    def _gather(self, unit: str, slot: int) -> None:
        u = self.s.units[unit]
        self._comm_after_compute()  # earlier readers of this window are enqueued
        if self.param_gate is not None and self.cuda:
            self.param_gate(unit, self.stream)
        with self._on_comm():
            # one partition (world 1, no forced collectives): DeepSpeed's gather returns
            # early, so the weights stay exact — no quantization round trip
            if self.quant and self.active:
                from . import kernels as K

                nb, w = K.quant_blocks(u.shard), self.world
                K.quant_int8(self.s.local_shard(self.s.shadow, unit), 1, self.q8_local[:u.shard],
                             self.qs_local[:nb])
                _all_gather(self.q8_all[:w * u.shard], self.q8_local[:u.shard], self.group, w)
                _all_gather(self.qs_all[:w * nb], self.qs_local[:nb], self.group, w)
                K.dequant_int8(self.q8_all[:w * u.shard], self.qs_all[:w * nb], w,
                               self.s.win_w[slot][:u.size])
            elif not self.s.alias_w:
                _all_gather(self.s.win_w[slot][:u.size], self.s.local_shard(self.s.shadow, unit),
                            self.group, self.world)
        self.w_ready[slot] = self._event()
        if self.res[slot] is not None:
            self.s.bound_w.pop(self.res[slot], None)
        self.res[slot] = unit
        self.stats["gathers"] += 1

    def _acquire(self, unit: str, order: list[str]) -> None:
        slot = self.res.index(unit) if unit in self.res else None
        if slot is None:
            slot = 0 if self.cur is None else 1 - self.cur
            self._gather(unit, slot)
        self._wait(self.w_ready[slot])
        self.cur = slot
        self.s.bound_w[unit] = slot
        i = order.index(unit)
        if i + 1 < len(order) and order[i + 1] not in self.res:
            self._gather(order[i + 1], 1 - slot)

    # ------------------------------------------------------------ replicate mode (ZeRO-2)
    def _gather_rep(self, unit: str) -> None:
        u = self.s.units[unit]
        self._comm_after_compute()
        if self.param_gate is not None and self.cuda:
            self.param_gate(unit, self.stream)
        with self._on_comm():
            _all_gather(self.s.rep_w[u.rep_lo:u.rep_lo + u.size],
                        self.s.local_shard(self.s.shadow, unit), self.group, self.world)
        self.rep_ready[unit] = self._event()
        self.stats["gathers"] += 1

    def _ensure(self, unit: str, order: list[str]) -> None:
        """replicate mode: a stale unit (updated by the last step) is gathered, waited for
        and re-transposed before use; the next stale unit's gather is issued behind it."""
        if unit in self.stale:
            if unit not in self.rep_ready:
                self._gather_rep(unit)
            self._wait(self.rep_ready.pop(unit))
            self.s.refresh_unit_transposed(unit)
            self.stale.discard(unit)
        i = order.index(unit)
        for nxt in order[i + 1:]:
            if nxt in self.stale:
                if nxt not in self.rep_ready:
                    self._gather_rep(nxt)
                break

    # ------------------------------------------------------------ fp32 units
    def _gather_f32(self, unit: str) -> None:
        """All-gather an fp32 unit's master shards (ZeRO-3: into the fp32 window; ZeRO-2: into
        its replicated fp32 copy) on the comm stream."""
        u = self.s.units[unit]
        self._comm_after_compute()  # earlier readers of the window are enqueued
        if self.param_gate is not None and self.cuda:
            self.param_gate(unit, self.stream)
        with self._on_comm():
            dst = (self.s.rep_f32[u.rep_lo:u.rep_lo + u.size] if self.replicate
                   else self.s.win_f32[:u.size])
            _all_gather(dst, self.s.local_shard(self.s.master, unit), self.group, self.world)
        self.f32_ready[unit] = self._event()
        if not self.replicate:
            self.s.bound_f32 = None  # the window is being overwritten
        self.stats["gathers"] += 1

    def _f32_needed(self, unit: str) -> bool:
        if self.replicate:
            return unit in self.stale
        return self.s.bound_f32 != unit

    def _acquire_f32(self, unit: str) -> None:
        if self._f32_needed(unit) and unit not in self.f32_ready:
            self._gather_f32(unit)
        if unit in self.f32_ready:
            self._wait(self.f32_ready.pop(unit))
            if self.replicate:
                self.stale.discard(unit)
        if not self.replicate:
            self.s.bound_f32 = unit

    def _prefetch_f32(self, unit: str) -> None:
        nxt = self.f32_next.get(unit)
        if nxt is not None and self._f32_needed(nxt) and nxt not in self.f32_ready:
            self._gather_f32(nxt)

    def forward(self, unit: str) -> None:
        if unit in self.f32:
            self._acquire_f32(unit)
            return
        if self.replicate:
            self._ensure(unit, self.fwd_order)
        else:
            self._acquire(unit, self.fwd_order)
        self._prefetch_f32(unit)

    def backward(self, unit: str) -> None:
        from . import kernels as K

        if unit in self.f32:  # the backward of an fp32 unit (embedding) reads no weights
            self.open_grad(unit)
            return
        if self.replicate:
            self._ensure(unit, self.bwd_order)
            self.open_grad(unit)
            return
        self._acquire(unit, self.bwd_order)
        if self.s.bound_wt != unit:
            self.s.bound_wt = unit
            for n in self.s.units[unit].offsets:
                if n in self.s.transposed:
                    K.transpose_bf16(self.s.w(n), self.s.wt(n))
        self.open_grad(unit)

    # ------------------------------------------------------------ gradients
    def open_grad(self, unit: str) -> None:
        if unit in self.s.bound_g:
            return
        if self.direct:
            self.s.bound_g[unit] = -1
            return
        used = set(self.s.bound_g.values())
        free = [k for k in (0, 1) if k not in used]
        if not free:
            raise RuntimeError("ZeRO-3: more than two gradient windows open")
        slot = min(free, key=lambda k: self.rs_seq[k])  # the longest-finished reduce-scatter
        self._wait(self.rs_done[slot])  # the previous reduce-scatter has read this window
        self.s.win_g[slot][:self.s.units[unit].size].zero_()
        self.s.bound_g[unit] = slot

    def backward_done(self, unit: str) -> None:
        slot = self.s.bound_g.pop(unit)
        u = self.s.units[unit]
        self._comm_after_grads()
        if slot < 0:  # direct: the gradient is in the shard already
            if self.final_pass and self.grad_final_hook is not None:
                self.grad_final_hook(u.local_lo, u.local_lo + u.shard, self.stream)
            self.stats["reduce_scatters"] += 1
            return
        with self._on_comm():
            tmp = self.rs_tmp[slot][:u.shard]
            if self.quant and self.active:
                from . import kernels as K

                nb, w = K.quant_blocks(u.shard), self.world
                K.quant_int4(self.s.win_g[slot][:u.size], w, self.q4_send[:w * u.shard // 2],
                             self.q4s_send[:w * nb])
                _all_to_all(self.q4_recv[:w * u.shard // 2], self.q4_send[:w * u.shard // 2],
                            self.group, w)
                _all_to_all(self.q4s_recv[:w * nb], self.q4s_send[:w * nb], self.group, w)
                tmp.zero_()
                K.dequant_int4_sum(self.q4_recv[:w * u.shard // 2], self.q4s_recv[:w * nb], w, tmp)
            elif not self.active:
                tmp.copy_(self.s.win_g[slot][:u.size])
            else:
                dist.reduce_scatter_tensor(tmp, self.s.win_g[slot][:u.size],
                                           op=dist.ReduceOp.SUM, group=self.group)
            self.s.local_shard(self.s.grad, unit).add_(tmp)
        self.rs_done[slot] = self._event()
        if self.final_pass and self.grad_final_hook is not None:
            self.grad_final_hook(u.local_lo, u.local_lo + u.shard, self.stream)
        self.stats["reduce_scatters"] += 1
        self.rs_seq[slot] = self.stats["reduce_scatters"]

    def reset(self) -> None:
        """Abandon an interrupted micro-batch (Engine.reset): wait for the comm stream,
        close every gradient window and forget the gathered units."""
        if self.cuda:
            self.stream.synchronize()
        self.s.bound_g.clear()
        self.rs_done = [None, None]
        self.f32_ready.clear()
        if self.replicate:
            # a unit whose gather was issued but not yet consumed is complete now (stream
            # synchronised): it stays stale and is re-gathered on its next use
            self.rep_ready.clear()
            return
        self.gather_params()

    # ------------------------------------------------------------ step level
    def begin_overlap(self) -> None:
        """(DDP only) — the ZeRO-3 exchange is always overlapped."""

    def reduce_grads(self) -> None:
        """End of the step: unit shards are reduced already; all-reduce the persistent
        (replicated) region's gradients."""
        self._comm_after_grads()
        with self._on_comm():
            if self.active:
                dist.all_reduce(self.s.grad[:self.s.fp32_end], op=dist.ReduceOp.SUM,
                                group=self.group)
        if self.cuda:
            cur = self._compute()
            COMM_TIMER.wait(cur, lambda: cur.wait_stream(self.stream))

    def global_sumsq(self, kernels) -> torch.Tensor:
        """Σg² over the whole model: partitioned units summed across ranks, the
        replicated region counted once."""
        dev = self.s.device
        part = torch.zeros(1, dtype=torch.float32, device=dev)
        rep = torch.zeros(1, dtype=torch.float32, device=dev)
        kernels.sumsq_f32(self.s.grad[self.s.fp32_end:], part)
        if self.s.fp32_end:
            kernels.sumsq_f32(self.s.grad[:self.s.fp32_end], rep)
        if self.active:
            dist.all_reduce(part, op=dist.ReduceOp.SUM, group=self.group)
        return part + rep

    def all_reduce_scalar(self, x: torch.Tensor) -> torch.Tensor:
        raise RuntimeError("ZeRO-3: use global_sumsq (the replicated region is counted once)")

    def gather_params(self) -> None:
        """After the sharded update: every gathered window is stale (replicate mode: every
        unit's full bf16 copy; each is all-gathered before its next use)."""
        self.f32_ready.clear()
        if self.replicate:
            self.stale = set(self.s.units)  # fp32 units included
            self.rep_ready.clear()
            return
        self.res = [None, None]
        self.cur = None
        self.s.bound_w.clear()
        self.s.bound_wt = None
        self.s.bound_f32 = None


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
