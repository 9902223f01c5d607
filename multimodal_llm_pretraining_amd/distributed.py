"""Data-parallel gradient / parameter exchange over RCCL (torch.distributed
backend "nccl" on ROCm = RCCL over xGMI), or gloo on CPU for tests.

Replaces DDP's bucketed all-reduce and DeepSpeed ZeRO-1/2's reduce-scatter +
all-gather (src/train.py:170-181) with collectives on the
ONE flat gradient / bf16-shadow buffer of params.ParamStore:

* ``ddp``   : all_reduce(SUM) of each layer's grads as soon as the last micro-batch's
  backward has produced them (overlapped with the rest of the backward), or of the
  flat fp32 grads in `bucket_mb` buckets;
* ``zero1``: (stage 1: no gradient partitioning, no overlap) one reduce_scatter(SUM) into
  the shards after the backward, then the sharded fused Adam + all_gather of the bf16
  shadow shards.
ZeRO-2 (stage 2: gradients partitioned too) is not here: it runs on zero3.py's per-unit
partition with replicated bf16 weights (Zero3Store(replicate=True)), so no rank holds a
full fp32 gradient or master buffer — DeepSpeed's memory semantics.

Gradients are pre-scaled by 1/num_items of the GLOBAL batch inside the loss
kernel, so a SUM reduction reproduces single-process semantics exactly.
Collectives run on a dedicated stream ordered after the backward by an event,
so an optional early launch (bucket ready) overlaps remaining backward work.
"""

from __future__ import annotations

import os

import torch
import torch.distributed as dist

MODES = ("ddp", "zero1")


class CommTimer:
    """Per-rank communication accounting for the multi-GPU bench line (off unless `on`):
    * busy    — HIP events on the communication stream around every exchange (the
      collectives and their staging copies): how long that stream is occupied;
    * exposed — events on the compute stream around each point where it WAITS for the
      communication stream (the end-of-backward join, a ZeRO gather the next unit needs):
      how long the step is stalled on communication that did not overlap compute."""

    def __init__(self):
        self.on = False
        self.busy: list = []
        self.exposed: list = []

    def _pair(self, stream):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        return e0, e1

    def span(self, stream):
        """context manager: events on `stream` around the enclosed enqueues"""
        timer = self

        class _Span:
            def __enter__(self_):
                if timer.on and stream is not None:
                    self_.ev = timer._pair(stream)
                return self_

            def __exit__(self_, *a):
                if timer.on and stream is not None:
                    self_.ev[1].record(stream)
                    timer.busy.append(self_.ev)
                return False
        return _Span()

    def wait(self, stream, fn) -> None:
        """run fn (a stream wait) bracketed by events on `stream` when on"""
        if not self.on or stream is None:
            fn()
            return
        e0, e1 = self._pair(stream)
        fn()
        e1.record(stream)
        self.exposed.append((e0, e1))

    def collect(self) -> dict:
        """totals (ms) since the last collect; the caller has synchronised the device"""
        busy = sum(a.elapsed_time(b) for a, b in self.busy)
        exposed = sum(a.elapsed_time(b) for a, b in self.exposed)
        out = {"comm_busy_ms": busy, "comm_exposed_ms": exposed, "comm_spans": len(self.busy),
               "comm_waits": len(self.exposed)}
        self.busy, self.exposed = [], []
        return out


COMM_TIMER = CommTimer()


def force_collectives() -> bool:
    """MMPT_FORCE_COLLECTIVES=1: run every collective even at world size 1 (no copy
    short-circuit) — exercises the RCCL path on a single GPU (tests/test_rccl_gpu.py)."""
    return os.environ.get("MMPT_FORCE_COLLECTIVES", "0") == "1" and dist.is_initialized()


def sharding_to_mode(sharding: str) -> str:
    """Map the reference's sharding strings (experiments/config.py:56-74,
    src/train.py:126-201) to the exchange mode implemented here."""
    return {
        "": "ddp",
        "zero_1": "zero1",
        "zero_2": "zero2",
        "fsdp_shard_grad_op": "zero2",
        "fsdp_hybrid_shard_zero2": "zero2",  # one node: the hybrid group is the node
        "zero_3": "zero3",
        "zero_3++": "zero3",  # + int8 weight gather / int4 grad all-to-all (Zero3Sync.quant)
        "fsdp_full_shard": "zero3",
        "fsdp_hybrid_shard": "zero3",
    }.get(sharding, "unsupported")


class GradSync:
    def __init__(self, grad: torch.Tensor, shadow: torch.Tensor | None, shard_size: int,
                 mode: str, group=None, bucket_mb: float = 256.0,
                 master: torch.Tensor | None = None, fp32_end: int = 0,
                 min_overlap_elems: int = 1 << 20, spans: list | None = None):
        """spans: sorted [lo, hi) of every parameter in the flat buffer."""
        if mode not in MODES:
            raise ValueError(f"mode {mode!r} not in {MODES}")
        self.grad, self.shadow, self.mode, self.group = grad, shadow, mode, group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.shard_size = shard_size
        # zero: the fp32 master of [0, fp32_end) is read directly by the step
        # (params.is_fp32_read) and must be re-synchronised after the sharded update
        self.master, self.fp32_end = master, fp32_end
        self.min_overlap_elems = min_overlap_elems
        if grad.numel() != shard_size * self.world:
            raise ValueError("flat buffer not divisible into world shards")
        elems = max(1, int(bucket_mb * 2**20) // grad.element_size())
        self.buckets = [(o, min(o + elems, grad.numel())) for o in range(0, grad.numel(), elems)]
        self.cuda = grad.is_cuda
        self.stream = torch.cuda.Stream(device=grad.device) if self.cuda else None
        self.force = force_collectives()
        # gloo has no CUDA `reduce`: emulate it with an all_reduce there (tests only)
        self._gloo = dist.is_initialized() and dist.get_backend(group) == "gloo"
        # overlap (ddp): ranges whose grads are final, already launched as async all-reduces
        self.overlap = False
        self.lazy_gather = False  # offload.ShardGather owns the post-step parameter gather
        self._works: list = []
        self._covered: list[tuple[int, int]] = []
        self.stats = {"overlapped": 0}
        self._spans = sorted(spans) if spans else [(0, grad.numel())]

    @property
    def _active(self) -> bool:
        return self.world > 1 or self.force

    # ---------------------------------------------------------------- overlap (ddp)
    def begin_overlap(self) -> None:
        """Arm the ready-hook for the LAST micro-batch of a step: from now on every
        on_ready(lo, hi) launches (ddp) an async all-reduce of grad[lo:hi] on RCCL's stream
        behind the backward kernels already queued."""
        self.overlap = self.mode == "ddp" and self._active
        self._works, self._covered = [], []

    def on_ready(self, lo: int, hi: int) -> None:
        if not self.overlap:
            return
        # tiny runs (LayerNorm γ/β) are left to the final sweep over uncovered ranges
        if hi - lo < self.min_overlap_elems:
            return
        # on the communication stream (ordered after the backward kernels queued so far):
        # the all-reduce runs beside the rest of the backward; reduce_grads joins it
        with self._on_comm():
            dist.all_reduce(self.grad[lo:hi], op=dist.ReduceOp.SUM, group=self.group)
        self._covered.append((lo, hi))
        self.stats["overlapped"] += 1

    def reset(self) -> None:
        """Abandon an interrupted step: finish the collectives already launched (every
        rank launched the same ones) and disarm the overlap."""
        for w in self._works:
            w.wait()
        self.overlap, self._works, self._covered = False, [], []

    def _uncovered(self) -> list[tuple[int, int]]:
        gaps, pos = [], 0
        for lo, hi in sorted(self._covered):
            if lo > pos:
                gaps.append((pos, lo))
            pos = max(pos, hi)
        if pos < self.grad.numel():
            gaps.append((pos, self.grad.numel()))
        return gaps

    def shard(self, buf: torch.Tensor) -> torch.Tensor:
        return self.shard_of(buf, self.rank)

    def shard_of(self, buf: torch.Tensor, r: int) -> torch.Tensor:
        return buf[r * self.shard_size:(r + 1) * self.shard_size]

    def _on_comm(self):
        if not self.cuda:
            return _Null()
        self.stream.wait_stream(torch.cuda.current_stream(self.grad.device))
        return _Comm(self.stream)

    def _join(self):
        if self.cuda:
            cur = torch.cuda.current_stream(self.grad.device)
            COMM_TIMER.wait(cur, lambda: cur.wait_stream(self.stream))

    def reduce_grads(self) -> None:
        """After the last micro-batch's backward: make the grads the global sum
        (ddp: everywhere; zero: on this rank's shard)."""
        if not self._active:
            return
        if self.overlap:
            with self._on_comm():
                for lo, hi in self._uncovered():  # padding / params never announced
                    dist.all_reduce(self.grad[lo:hi], op=dist.ReduceOp.SUM, group=self.group)
            for w in self._works:
                w.wait()
            self._join()  # the compute stream waits for every overlapped all-reduce
            self.overlap, self._works, self._covered = False, [], []
            return
        with self._on_comm():
            if self.mode == "ddp":
                for lo, hi in self.buckets:
                    dist.all_reduce(self.grad[lo:hi], op=dist.ReduceOp.SUM, group=self.group)
            else:
                out = self.shard(self.grad)
                tmp = torch.empty_like(out)
                dist.reduce_scatter_tensor(tmp, self.grad, op=dist.ReduceOp.SUM, group=self.group)
                out.copy_(tmp)
        self._join()

    def all_reduce_scalar(self, x: torch.Tensor) -> torch.Tensor:
        if self._active:
            dist.all_reduce(x, op=dist.ReduceOp.SUM, group=self.group)
        return x

    def _global(self, r: int) -> int:
        return dist.get_global_rank(self.group, r) if self.group is not None else r

    def gather_params(self) -> None:
        """zero: every rank updated only its shard of the bf16 shadow → all-gather (under
        the overlapped offload the trainer's offload.ShardGather does it per chunk, lazily)."""
        if not self._active or self.mode == "ddp" or self.shadow is None or self.lazy_gather:
            return
        with self._on_comm():
            src = self.shard(self.shadow).clone()
            dist.all_gather_into_tensor(self.shadow, src, group=self.group)
            if self.master is not None:  # fp32-read region: broadcast from its owners
                for r in range(self.world):
                    lo = r * self.shard_size
                    hi = min(lo + self.shard_size, self.fp32_end)
                    if hi <= lo:
                        break
                    src_rank = dist.get_global_rank(self.group, r) if self.group is not None else r
                    dist.broadcast(self.master[lo:hi], src=src_rank, group=self.group)
        self._join()


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class _Comm:
    """`with torch.cuda.stream(comm)` + CommTimer's busy span on that stream"""

    def __init__(self, stream):
        self.ctx, self.span = torch.cuda.stream(stream), COMM_TIMER.span(stream)

    def __enter__(self):
        self.ctx.__enter__()
        self.span.__enter__()
        return self

    def __exit__(self, *a):
        self.span.__exit__(*a)
        return self.ctx.__exit__(*a)
