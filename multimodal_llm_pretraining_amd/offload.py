"""Optimizer-state offload to host memory (DeepSpeed ZeRO-Offload / FSDP CPUOffload,
selected by the reference's `offloading` knob: experiments/config.py:68-74 →
TrainingClass.zero_offload_optimizer / zero_offload_params / fsdp_offload →
src/train.py:182-213).

The rank's optimizer range (the whole model under DDP, its 1/N shard under ZeRO) keeps
its fp32 master, Adam m and v in pinned host memory; the HBM keeps the bf16 shadow the
step reads, the fp32 gradients and the fp32-read region.  One optimizer step:

  grad shard  --D2H (pinned, copy stream)-->  host
  CPU Adam(W) (libmmpt_host.so, OpenMP, writes fp32 master + bf16 copy)
  bf16 shard  --H2D (second copy stream)-->  HBM shadow;  fp32-read part --H2D--> HBM master

pipelined over 64-MiB chunks: while the host updates chunk i, chunk i+1's gradients are
still coming down and chunk i-1's bf16 parameters going up (PCIe is full duplex), so the
step costs ≈ max(D2H, host Adam, H2D) rather than their sum.  Same arithmetic as one
whole-range call.

Overlapped mode (`async_update`, the default where the post-step parameter exchange is
local: DDP, ZeRO-3, or ZeRO-1/2 without an active collective):

* gradient ranges announced final during the LAST micro-batch's backward (`grad_final`:
  a unit's reduce-scatter under ZeRO-3, a layer group's grads at world 1) start their D2H
  at once, under the rest of the backward;
* `step` downloads what is left, lets the compute stream zero the gradients once every
  download has landed, and hands the chunks to a host worker thread (ctypes releases the
  GIL) — the call returns without waiting for the update;
* the flat range is laid out in forward order (fp32-read region, ViT, projector, text
  layers, lm_head), so the worker finishes the chunks in the order the next forward needs
  them: `wait_range(lo, hi, stream)` makes a stream wait for just the chunks covering a
  unit (the engine's residency hook calls it per unit), and the host update of step t
  runs under the forward of step t+1 (DeepSpeed ZeRO-Offload's one-step overlap without
  its stale-parameter delay: every unit still sees its updated weights);
* `join()` completes the update (timing harnesses, checkpoints, the next `step`).

Gradient clipping uses the device Σg² (already reduced across ranks) — the coefficient
is read back once per step.  There is no device fallback: a missing libmmpt_host.so
raises.
"""

from __future__ import annotations

import ctypes
import os
import threading
from ctypes import c_double, c_float, c_int, c_int64, c_void_p

import torch

from .optim import AdamConfig

_HERE = os.path.dirname(os.path.abspath(__file__))
HOST_LIB_PATH = os.environ.get("MMPT_HOST_LIB") or os.path.join(_HERE, "lib", "libmmpt_host.so")
HOST_ABI_VERSION = 1

HOST_SIGNATURES = {
    "mmpt_host_abi_version": (c_int, []),
    "mmpt_host_last_error": (ctypes.c_char_p, []),
    "mmpt_host_adam_step": (c_int, [c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_float, c_float, c_float, c_float, c_float, c_int, c_int64,
                                    c_void_p, c_int]),
    "mmpt_host_sumsq": (c_int, [c_int64, c_void_p, ctypes.POINTER(c_double), c_int]),
    "mmpt_host_simd_width": (c_int, []),
}

_hlib = None


def load_host() -> ctypes.CDLL:
    global _hlib
    if _hlib is not None:
        return _hlib
    if not os.path.exists(HOST_LIB_PATH):
        raise RuntimeError(f"libmmpt_host.so not found at {HOST_LIB_PATH}: build with "
                           "make -C multimodal_llm_pretraining_amd/csrc")
    lib = ctypes.CDLL(HOST_LIB_PATH)
    for name, (res, args) in HOST_SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    if lib.mmpt_host_abi_version() != HOST_ABI_VERSION:
        raise RuntimeError("libmmpt_host.so ABI mismatch; rebuild")
    _hlib = lib
    return lib


def _host_threads() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))


def host_adam_step(p, g, m, v, pb, *, lr, beta1, beta2, eps, weight_decay, adamw, step,
                   grad_scale=None, threads=0) -> None:
    """CPU Adam(W) over contiguous fp32 CPU tensors (pb: int16/bf16 CPU tensor or None)."""
    lib = load_host()
    for t in (p, g, m, v):
        if t.device.type != "cpu" or t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError("host_adam_step: fp32 contiguous CPU tensors expected")
    gs = None
    if grad_scale is not None:
        gs_t = torch.tensor([float(grad_scale)], dtype=torch.float32)
        gs = gs_t.data_ptr()
    rc = lib.mmpt_host_adam_step(p.numel(), p.data_ptr(), g.data_ptr(), m.data_ptr(),
                                 v.data_ptr(), None if pb is None else pb.data_ptr(), lr, beta1,
                                 beta2, eps, weight_decay, int(adamw), step, gs,
                                 threads or _host_threads())
    if rc != 0:
        raise RuntimeError("mmpt_host_adam_step: " + lib.mmpt_host_last_error().decode())


class HostAdam:
    """FusedAdam's interface (grad_sumsq / step / state_dict) with the optimizer range in
    host memory.  `device_master` + `fp32_end`: the first `fp32_end` elements of this
    rank's range are read by the step from the fp32 master on the device and are copied
    back after each update."""

    def __init__(self, params: torch.Tensor, grads: torch.Tensor, shadow: torch.Tensor | None,
                 cfg: AdamConfig, device_master: torch.Tensor | None = None, fp32_end: int = 0,
                 async_update: bool = False):
        load_host()
        self.dev_p, self.g, self.shadow, self.cfg = params, grads, shadow, cfg
        self.fp32_end = fp32_end
        pin = params.is_cuda
        n = params.numel()
        # the host master is taken from the device master at the first step (so a
        # store.load() after construction is honoured); from then on it is authoritative
        self.p = torch.empty(n, dtype=torch.float32, pin_memory=pin)
        self._initialised = False
        self.m = torch.zeros(n, dtype=torch.float32, pin_memory=pin)
        self.v = torch.zeros(n, dtype=torch.float32, pin_memory=pin)
        self.g_host = torch.empty(n, dtype=torch.float32, pin_memory=pin)
        self.pb_host = torch.empty(n, dtype=torch.bfloat16, pin_memory=pin)
        self.step_count = 0
        self._sumsq = torch.zeros(1, dtype=torch.float32, device=grads.device)
        self._coef = torch.ones(1, dtype=torch.float32, device=grads.device)
        self.chunk = int(os.environ.get("MMPT_OFFLOAD_CHUNK", str(1 << 24)))  # elements
        if self.g.is_cuda:
            self.d2h = torch.cuda.Stream(device=grads.device)
            self.h2d = torch.cuda.Stream(device=grads.device)
        self.async_update = bool(async_update) and self.g.is_cuda
        self._pref: list = []         # (lo, hi, event): downloads issued during the backward
        self._worker: threading.Thread | None = None
        self._bounds: list = []       # chunks of the update in flight
        self._done: list = []         # per chunk: threading.Event (H2D enqueued)
        self._h2d_ev: list = []       # per chunk: cuda Event (H2D complete)
        self._err: BaseException | None = None
        self.stats = {"prefetched_elems": 0, "waits": 0}
        # release(host_p) -> new device master view of this range's first fp32_end elements:
        # called once the host master is initialised, to free the device fp32 master (the
        # trainer wires it when it owns the store; DeepSpeed's optimizer offload keeps no
        # fp32 master on the device)
        self.release = None
        self.released = False

    def init_host(self) -> None:
        """Take the host master from the device master (once), then release the device
        copy if a release hook is wired.  Called by the first step, or right away by a
        trainer whose store already holds the initial weights."""
        if self._initialised:
            return
        self.p.copy_(self.dev_p.detach())
        self._initialised = True
        if self.release is not None and os.environ.get("MMPT_OFFLOAD_KEEP_MASTER", "0") != "1":
            self.dev_p = self.release(self.p)
            self.released = True
            if self.g.is_cuda:
                torch.cuda.empty_cache()

    def grad_sumsq(self) -> torch.Tensor:
        from . import kernels as K

        K.sumsq_f32(self.g, self._sumsq)
        return self._sumsq

    # ---------------------------------------------------------------- overlap
    def _chunks(self, lo: int, hi: int) -> list[int]:
        return [i for i, (a, b) in enumerate(self._bounds) if a < hi and lo < b]

    def wait_range(self, lo: int, hi: int, stream) -> None:
        """Make `stream` wait until the host update of [lo, hi) is back on the device."""
        if self._worker is None:
            return
        for i in self._chunks(lo, hi):
            if not self._done[i].is_set():
                self.stats["waits"] += 1
                self._done[i].wait()
            if self._err is not None:
                self.join()  # re-raises
            stream.wait_event(self._h2d_ev[i])

    def join(self) -> None:
        """Finish the update in flight (host side and its H2D on the compute stream)."""
        if self._worker is None:
            return
        self._worker.join()
        self._worker = None
        err, self._err = self._err, None
        torch.cuda.current_stream(self.g.device).wait_stream(self.h2d)
        if err is not None:
            raise RuntimeError("host Adam worker failed") from err

    def grad_final(self, lo: int, hi: int, stream=None) -> None:
        """g[lo:hi] is final once the work queued on `stream` (default: the current stream)
        completes: start its download now (last micro-batch of a step only)."""
        if not self.g.is_cuda or hi <= lo:
            return
        self.join()  # g_host may still be read by the previous step's update
        self.d2h.wait_stream(stream if stream is not None else
                             torch.cuda.current_stream(self.g.device))
        with torch.cuda.stream(self.d2h):
            self.g_host[lo:hi].copy_(self.g[lo:hi], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.d2h)
        self._pref.append((lo, hi, ev))
        self.stats["prefetched_elems"] += hi - lo

    def _update(self, bounds, landed, kw) -> None:
        """Chunks in order: wait for their gradients, CPU Adam, H2D (shadow + fp32 part)."""
        try:
            with torch.cuda.device(self.g.device):
                for i, (lo, hi) in enumerate(bounds):
                    for ev in landed[i]:
                        ev.synchronize()
                    host_adam_step(self.p[lo:hi], self.g_host[lo:hi], self.m[lo:hi],
                                   self.v[lo:hi], self.pb_host[lo:hi], **kw)
                    with torch.cuda.stream(self.h2d):
                        if self.shadow is not None:
                            self.shadow[lo:hi].copy_(self.pb_host[lo:hi], non_blocking=True)
                        f_hi = min(hi, self.fp32_end)
                        if f_hi > lo:
                            self.dev_p[lo:f_hi].copy_(self.p[lo:f_hi], non_blocking=True)
                        ev = torch.cuda.Event()
                        ev.record(self.h2d)
                    self._h2d_ev[i] = ev
                    self._done[i].set()
        except BaseException as e:  # surfaced by join()/wait_range()
            self._err = e
            for d in self._done:
                d.set()

    def step(self, lr: float, sumsq: torch.Tensor | None = None) -> None:
        from . import kernels as K

        c = self.cfg
        self.join()
        self.init_host()
        self._rerelease()
        self.step_count += 1
        scale = None
        if c.max_grad_norm and c.max_grad_norm > 0:
            if sumsq is None:
                sumsq = self.grad_sumsq()
            K.clip_coef(sumsq, c.max_grad_norm, self._coef)
            scale = float(self._coef.item())
        kw = dict(lr=lr, beta1=c.betas[0], beta2=c.betas[1], eps=c.eps,
                  weight_decay=c.weight_decay, adamw=c.adamw, step=self.step_count,
                  grad_scale=scale)
        if not self.g.is_cuda:
            self.g_host.copy_(self.g)
            host_adam_step(self.p, self.g_host, self.m, self.v, self.pb_host, **kw)
            if self.shadow is not None:
                self.shadow.copy_(self.pb_host)
            if self.fp32_end:
                self.dev_p[:self.fp32_end].copy_(self.p[:self.fp32_end])
            return
        n = self.p.numel()
        bounds = [(o, min(o + self.chunk, n)) for o in range(0, n, self.chunk)]
        cur = torch.cuda.current_stream(self.g.device)
        self.d2h.wait_stream(cur)  # the gradients (and the clip coefficient) are final
        self.h2d.wait_stream(cur)
        # download every piece of each chunk not already on its way (grad_final)
        pref, self._pref = self._pref, []
        landed = []
        with torch.cuda.stream(self.d2h):
            for lo, hi in bounds:
                evs = [ev for a, b, ev in pref if a < hi and lo < b]
                pos = lo
                for a, b in sorted((max(a, lo), min(b, hi)) for a, b, _ in pref
                                   if a < hi and lo < b) + [(hi, hi)]:
                    if a > pos:
                        self.g_host[pos:a].copy_(self.g[pos:a], non_blocking=True)
                    pos = max(pos, b)
                ev = torch.cuda.Event()
                ev.record(self.d2h)
                landed.append(evs + [ev])
        self._bounds = bounds
        self._done = [threading.Event() for _ in bounds]
        self._h2d_ev = [None] * len(bounds)
        if not self.async_update:
            self._worker = None
            self._update(bounds, landed, kw)
            if self._err is not None:
                err, self._err = self._err, None
                raise RuntimeError("host Adam failed") from err
            cur.wait_stream(self.h2d)
            return
        # the compute stream may zero the gradients once they are all on the host
        cur.wait_stream(self.d2h)
        self._worker = threading.Thread(target=self._update, args=(bounds, landed, kw),
                                        name="mmpt-host-adam", daemon=True)
        self._worker.start()

    def sync_master(self) -> None:
        """Copy the (authoritative) host master of this rank's range back to the device
        master buffer — for checkpoints / inspection, not part of the step.  A released
        device master is re-materialised first (restore_hook); the release hook stays wired,
        so the next `step` frees it again (`_rerelease`)."""
        self.join()
        if not self._initialised:
            return
        if self.released:
            self.dev_p = self.restore_hook()
            self.released = False
        self.dev_p.copy_(self.p)

    def _rerelease(self) -> None:
        """After a sync_master: hand the device fp32 master back (the host copy stayed
        authoritative; the kept region on the device is current)."""
        if (self._initialised and not self.released and self.release is not None
                and os.environ.get("MMPT_OFFLOAD_KEEP_MASTER", "0") != "1"):
            self.dev_p = self.release(self.p)
            self.released = True
            if self.g.is_cuda:
                torch.cuda.empty_cache()

    def state_dict(self) -> dict:
        self.join()
        return {"m": self.m, "v": self.v, "step": self.step_count}


class ShardGather:
    """ZeRO-1 under the overlapped offload at world > 1: the bf16 shadow all-gather after the
    sharded update, cut into the host update's chunks (HostAdam bounds, this rank's local
    coordinates) and issued lazily: before a unit's first forward, every chunk index that
    covers the unit on ANY rank's shard is gathered (ascending chunk order — the same
    sequence of collectives on every rank), each one on the communication stream right after
    this rank's host update of that chunk has been uploaded.  The fp32-read region's master
    is broadcast from its owners the same way.  (The synchronous path all-gathers the whole
    shadow at once after the update.)"""

    def __init__(self, store, opt: HostAdam, sync):
        self.s, self.opt, self.sync = store, opt, sync
        self.S, self.world, self.rank = store.shard_size, sync.world, sync.rank
        self.done: dict[int, object] = {}
        self.region_done = False

    def chunks_for(self, lo: int, hi: int) -> list[int]:
        """chunk indices (local bounds) overlapping global [lo, hi) on any rank's shard"""
        out = set()
        for r in range(self.world):
            a, b = max(lo - r * self.S, 0), min(hi - r * self.S, self.S)
            if a < b:
                out.update(i for i, (c0, c1) in enumerate(self.opt._bounds) if c0 < b and a < c1)
        return sorted(out)

    def _gather(self, i: int) -> None:
        import torch.distributed as dist

        a, b = self.opt._bounds[i]
        sh, S, w = self.s.shadow, self.S, self.world
        comm = self.sync.stream
        comm.wait_stream(torch.cuda.current_stream(sh.device))
        self.opt.wait_range(a, b, comm)  # this rank's chunk i is back on the device
        with self.sync._on_comm():
            tmp = torch.empty(w * (b - a), dtype=sh.dtype, device=sh.device)
            dist.all_gather_into_tensor(tmp, sh[self.rank * S + a:self.rank * S + b].clone(),
                                        group=self.sync.group)
            for r in range(w):
                if r != self.rank:
                    sh[r * S + a:r * S + b].copy_(tmp[r * (b - a):(r + 1) * (b - a)])
            ev = torch.cuda.Event()
            ev.record(comm)
        self.done[i] = ev

    def ensure(self, lo: int, hi: int, stream) -> None:
        for i in self.chunks_for(lo, hi):
            if i not in self.done:
                self._gather(i)
        for i in self.chunks_for(lo, hi):
            stream.wait_event(self.done[i])

    def region(self, region_end: int, stream) -> None:
        """the fp32-read region: shadow chunks + the master broadcast from its owners"""
        import torch.distributed as dist

        self.ensure(0, region_end, stream)
        if self.region_done or self.sync.master is None:
            return
        comm = self.sync.stream
        for r in range(self.world):
            lo, hi = r * self.S, min((r + 1) * self.S, region_end)
            if hi <= lo:
                break
            if r == self.rank:  # its fp32 part is uploaded with the chunks covering it
                self.opt.wait_range(0, hi - lo, comm)
            with self.sync._on_comm():
                dist.broadcast(self.sync.master[lo:hi], src=self.sync._global(r),
                               group=self.sync.group)
        ev = torch.cuda.Event()
        ev.record(comm)
        stream.wait_event(ev)
        self.region_done = True

    def arm(self) -> None:
        self.done, self.region_done = {}, False


class OffloadGate:
    """The engine's residency hook (`Engine.units`) for the non-ZeRO-3 stores under the
    overlapped offload: before a unit's first forward after a step, the compute stream
    waits for the host update of that unit's parameters (ZeRO-1 at world > 1: for the
    ShardGather of those parameters) and the unit's transposed bf16 weights are rebuilt from
    the new shadow (ParamStore.refresh_transposed, per unit)."""

    def __init__(self, store, opt: HostAdam, region_end: int, gather: ShardGather | None = None):
        from .zero3 import unit_of

        self.s, self.opt, self.region_end = store, opt, region_end
        self.gather = gather
        self.ranges: dict[str, list[int]] = {}
        self.region_t: list[str] = []
        self.trans: dict[str, list[str]] = {}
        for n, o in store.offsets.items():
            try:
                u = unit_of(n)
            except KeyError:
                u = None
            if u is None:  # fp32-read region
                if n in store.transposed:
                    self.region_t.append(n)
                continue
            hi = o + store.g(n).numel()
            r = self.ranges.setdefault(u, [o, hi])
            r[0], r[1] = min(r[0], o), max(r[1], hi)
            if n in store.transposed:
                self.trans.setdefault(u, []).append(n)
        self.stale: set[str] = set()
        self.region_stale = False

    def arm(self) -> None:
        """After an optimizer step: every unit waits for (and re-transposes) its update."""
        self.stale = set(self.ranges)
        self.region_stale = True
        if self.gather is not None:
            self.gather.arm()

    def _wait(self, lo: int, hi: int) -> None:
        cur = torch.cuda.current_stream(self.s.device)
        if self.gather is not None:
            self.gather.ensure(lo, hi, cur)
        else:
            self.opt.wait_range(lo, hi, cur)

    def region(self) -> None:
        """Before a forward: the fp32-read region (embeddings, LayerNorm) is current."""
        if not self.region_stale:
            return
        from . import kernels as K

        if self.gather is not None:
            self.gather.region(self.region_end, torch.cuda.current_stream(self.s.device))
        else:
            self.opt.wait_range(0, self.region_end, torch.cuda.current_stream(self.s.device))
        for n in self.region_t:
            K.transpose_bf16(self.s.w(n), self.s.wt(n))
        self.region_stale = False

    def forward(self, unit: str) -> None:
        if unit not in self.stale:
            return
        from . import kernels as K

        lo, hi = self.ranges[unit]
        self._wait(lo, hi)
        for n in self.trans.get(unit, []):
            K.transpose_bf16(self.s.w(n), self.s.wt(n))
        self.stale.discard(unit)

    def backward(self, unit: str) -> None:
        self.forward(unit)  # (a backward without a forward since the step: never in practice)

    def backward_done(self, unit: str) -> None:
        pass

    def open_grad(self, unit: str) -> None:
        pass

    def reset(self) -> None:
        pass
