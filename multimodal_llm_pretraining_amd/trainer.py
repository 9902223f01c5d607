"""ManualTrainer equivalent for the MI355X step (src/benchmarking/utils.py:40-80).

`manual_training_step(batch)` = one micro-batch forward + backward (the
reference's `Trainer.training_step`, gradients accumulate);
`manual_optimization_step()` = gradient exchange (DDP all-reduce or ZeRO
reduce-scatter) → clip (if max_grad_norm > 0) → fused Adam(W) → parameter
all-gather (ZeRO) → LR-scheduler step → zero_grad.

Loss normalisation follows HF Trainer's `num_items_in_batch` path: the CE sum
of every micro-batch of every rank is divided by the number of label tokens of
the whole global batch, so DP + gradient accumulation reproduce the
single-process step exactly.
"""

from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist

from . import config as C
from . import kernels as K
from .distributed import GradSync, sharding_to_mode
from .engine import Batch, Engine
from .optim import AdamConfig, AdamOverlap, FusedAdam, Schedule
from .params import ParamStore, init_normal
from .zero3 import Zero3Store, Zero3Sync


@dataclass
class StepConfig:
    model: str = "vit-b16-pythia-1b"
    micro_batch_size: int = 1
    grad_accum: int = 1
    sharding: str = ""  # "", zero_1, zero_2, zero_3, fsdp_shard_grad_op, fsdp_full_shard, ...
    activation_checkpointing: bool = False
    offload: bool = False  # optimizer state (fp32 master, m, v) in host memory, CPU Adam
    seed: int = 0
    scheduler: str = "cosine"
    num_warmup_steps: int = 0
    num_training_steps: int = 1
    min_lr_rate: float = 0.0


class ManualTrainer:
    def __init__(self, step_cfg: StepConfig, adam: AdamConfig, device: torch.device | str = "cuda",
                 model_cfg: C.ModelConfig | None = None, group=None,
                 store: ParamStore | None = None, engine: Engine | None = None,
                 init: bool = True):
        """`store`/`engine`: adopt existing ones (e.g. those of models.MMPTForPretraining)
        instead of building and initialising new ones.  init=False: a new store is left
        zeroed (the caller loads weights into it)."""
        self.step_cfg = step_cfg
        self.cfg = model_cfg or C.get_config(step_cfg.model)
        self.device = torch.device(device)
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        mode = sharding_to_mode(step_cfg.sharding)
        if mode == "unsupported":
            raise NotImplementedError(f"sharding {step_cfg.sharding!r} not implemented yet")
        if self.cfg.freeze_tower_and_llm and (mode != "ddp" or step_cfg.offload):
            raise NotImplementedError("freeze_tower_and_llm trains the projector only (6.3 M "
                                      "parameters): data parallel without sharding/offload")
        if mode == "zero3" and self.cfg.text.tie_embeddings:
            raise NotImplementedError("ZeRO-3 with a tied lm_head (Llama) is not implemented")
        # ZeRO-2 and ZeRO-3 share the per-unit partition (zero3.py): ZeRO-2 keeps the bf16
        # weights replicated, ZeRO-3 gathers them per use
        self.unit_mode = mode in ("zero2", "zero3") and not self.cfg.freeze_tower_and_llm
        own_store = store is None  # (a store adopted from the drop-in module backs its
        # nn.Parameters: its device master is never released)
        if store is None:
            if self.unit_mode:
                # DeepSpeed stage3_param_persistence_threshold "auto" = 10 x hidden
                # (src/train.py:182-194; tf:integrations/deepspeed.py): the fp32-read
                # parameters above it (token / position embeddings) are partitioned too.
                # A tied embedding (Llama) stays persistent: the lm_head reads its bf16
                # transpose.
                thr = None if self.cfg.text.tie_embeddings else 10 * self.cfg.text.hidden
                store = Zero3Store(C.param_shapes(self.cfg), self.device, self.world, self.rank,
                                   replicate=mode == "zero2", persist_threshold=thr)
            else:
                store = ParamStore(C.param_shapes(self.cfg), self.device, world=self.world,
                                   trainable=self.cfg.trainable if self.cfg.freeze_tower_and_llm
                                   else None)
            if init:
                init_normal(store, step_cfg.seed, cfg=self.cfg)
        elif store.world != self.world:
            raise ValueError(f"store laid out for world {store.world}, process group has {self.world}")
        elif self.unit_mode != isinstance(store, Zero3Store) or (
                self.unit_mode and store.replicate != (mode == "zero2")):
            raise ValueError("ZeRO-2/3 need a Zero3Store (replicate=True for ZeRO-2), and only "
                             "they use one")
        self.store = store
        self.engine = engine if engine is not None else Engine(self.cfg, self.store)
        self.engine.checkpointing = step_cfg.activation_checkpointing
        if self.unit_mode:
            self.sync = Zero3Sync(self.store, self.engine.unit_order(), group,
                                  quant=step_cfg.sharding == "zero_3++")
            self.engine.units = self.sync
            p, g, sh = self.store.master, self.store.grad, self.store.shadow
        elif self.cfg.freeze_tower_and_llm:
            # only the projector trains (src/models/llava.py:49-52): the optimizer and the
            # gradient exchange cover its contiguous range of the flat buffers, nothing else
            lo, hi = self._trainable_range()
            self.sync = GradSync(self.store.grad[lo:hi], self.store.shadow[lo:hi],
                                 (hi - lo) // self.world, mode, group)
            p, g, sh = self.store.master[lo:hi], self.store.grad[lo:hi], self.store.shadow[lo:hi]
        else:
            spans = [(o, o + self.store.g(n).numel()) for n, o in self.store.offsets.items()]
            self.sync = GradSync(self.store.grad, self.store.shadow, self.store.shard_size, mode,
                                 group, master=self.store.master, fp32_end=self.store.fp32_end,
                                 spans=spans)
            self.engine.grad_ready_hook = self.sync.on_ready
            if mode == "ddp":
                p, g, sh = self.store.master, self.store.grad, self.store.shadow
            else:
                p, g, sh = (self.sync.shard(self.store.master), self.sync.shard(self.store.grad),
                            self.sync.shard(self.store.shadow))
        self._gate = None
        self._pending_refresh = None
        self._offload_final = False
        if step_cfg.offload:
            from .offload import HostAdam, OffloadGate

            # overlapped update (offload.py) where the post-step parameter exchange is
            # local: the next forward gates per unit on the host update instead of waiting
            # for all of it (ZeRO-1/2 with an active all-gather need the whole shard)
            async_ok = (os.environ.get("MMPT_OFFLOAD_ASYNC", "1") != "0" and
                        self.device.type == "cuda")
            self.opt = HostAdam(p, g, sh, adam, device_master=self.store.master,
                                fp32_end=self.store.fp32_keep if self.unit_mode else
                                _fp32_overlap(self.store, self.sync, mode),
                                async_update=async_ok)
            if async_ok:
                if self.unit_mode:
                    self.sync.param_gate = lambda u, stream: self.opt.wait_range(
                        self.store.units[u].local_lo,
                        self.store.units[u].local_lo + self.store.units[u].shard, stream)
                    self.sync.grad_final_hook = self.opt.grad_final
                    self._region_end = self.store.fp32_end
                elif self.engine.units is None:
                    gather = None
                    if self.sync._active and mode == "zero1":  # per-chunk lazy all-gather
                        from .offload import ShardGather

                        gather = ShardGather(self.store, self.opt, self.sync)
                        self.sync.lazy_gather = True
                    self._gate = OffloadGate(self.store, self.opt, self.store.fp32_end, gather)
                    self.engine.units = self._gate
                    if not self.sync._active:  # world 1: grads are final as produced
                        hook = self.engine.grad_ready_hook

                        def ready(lo, hi, _hook=hook):
                            if _hook is not None:
                                _hook(lo, hi)
                            if self._offload_final:
                                self.opt.grad_final(lo, hi)
                        self.engine.grad_ready_hook = ready
            if own_store:
                self._wire_master_release(mode)
                if init:  # the initial weights are in place: move the master to the host now
                    self.opt.init_host()
        else:
            self.opt = FusedAdam(p, g, sh, adam)
        # the optimizer step overlapped with the next forward, per parameter unit
        # (optim.AdamOverlap): the flat data-parallel / single-GPU store
        self.adam_overlap = None
        if (not step_cfg.offload and mode == "ddp" and not self.unit_mode and
                not self.cfg.freeze_tower_and_llm and self.engine.units is None and
                self.device.type == "cuda" and isinstance(self.store, ParamStore) and
                os.environ.get("MMPT_ADAM_OVERLAP", "0") == "1"):
            self.adam_overlap = AdamOverlap(self.store, self.opt, self.engine.unit_order())
            self.engine.units = self.adam_overlap
        self.sched = Schedule(adam.lr, step_cfg.scheduler, step_cfg.num_warmup_steps,
                              step_cfg.num_training_steps, step_cfg.min_lr_rate)
        self.mode = mode
        # DDP: all-reduce each layer's grads as soon as the last micro-batch's backward
        # has produced them; ZeRO-2: reduce each shard to its owner as soon as all its
        # grads are final (both overlap the rest of the backward). ZeRO-1 (DeepSpeed
        # stage 1 has no overlap_comm) reduce-scatters once after the backward.
        self.overlap_comm = (mode == "ddp" and self.sync._active
                             and not self.cfg.freeze_tower_and_llm)
        # weights the optimizer changes (their transposed shadows are refreshed per step;
        # ZeRO-2/3 rebuild a unit's transposes when its new weights arrive — only the
        # replicated region's, the tied embedding, are refreshed here)
        self._refresh = None if not self.cfg.freeze_tower_and_llm else \
            [n for n in self.store.transposed if self.cfg.trainable(n)]
        if self.unit_mode:

            self._refresh = [n for n in self.store.transposed if self.store.unit_of(n) is None]

    def _wire_master_release(self, mode: str) -> None:
        """Offload: once the host master exists, free the device fp32 master except the
        region the step reads as fp32 (DeepSpeed offload_optimizer keeps the fp32 master
        in host memory only, src/train.py:203-207): 12 B/param of optimizer state leave the
        device instead of 8."""
        st, opt = self.store, self.opt
        if self.unit_mode:  # the persistent region + the fp32 units' shards
            keep, lo = st.fp32_keep, 0
        elif mode == "ddp":
            keep, lo = st.fp32_end, 0
        else:  # zero1: this rank's range starts at its shard
            keep, lo = st.fp32_end, self.sync.rank * st.shard_size

        def release(host_p, _st=st, _keep=keep, _lo=lo):
            new = _st.release_master(_keep, host_p, _lo)
            if isinstance(self.sync, GradSync) and self.sync.master is not None:
                self.sync.master = new
            # this range's device view: its part of the kept region (empty past it)
            return new[_lo:_lo + host_p.numel()] if _lo < _keep else new[:0]

        def restore(_st=st, _lo=lo):
            full = _st.restore_master()
            if isinstance(self.sync, GradSync) and self.sync.master is not None:
                self.sync.master = full
            n = opt.p.numel()
            return full[_lo:_lo + n]
        opt.release, opt.restore_hook = release, restore

    def _trainable_range(self) -> tuple[int, int]:
        """[lo, hi) of the flat buffers holding every trainable parameter (they are laid out
        contiguously, ParamStore(trainable=...)), widened to a multiple of 64·world
        elements — checked AFTER the widening, so the range never reaches a frozen
        parameter (FusedAdam / the all-reduce would otherwise touch it)."""
        names = [n for n in self.store.shapes if self.cfg.trainable(n)]
        lo = min(self.store.offsets[n] for n in names)
        hi = max(self.store.offsets[n] + self.store.g(n).numel() for n in names)
        q = 64 * self.world
        hi = lo + -(-(hi - lo) // q) * q
        frozen = [n for n in self.store.shapes if n not in names]
        if any(self.store.offsets[n] < hi and lo < self.store.offsets[n] + self.store.g(n).numel()
               for n in frozen):
            raise RuntimeError("the trainable range overlaps a frozen parameter (build the store "
                               "with ParamStore(trainable=cfg.trainable))")
        if hi > self.store.padded:
            raise RuntimeError("trainable range runs past the flat buffer")
        return lo, hi

    def stage(self, batch: dict, stream=None) -> Batch:
        """The device side of `_prepare_inputs`: host (ideally pinned) tensors are copied
        asynchronously and the index bookkeeping is built without a device sync; with
        `stream` the staging runs on that copy stream, overlapped with the step."""
        return Batch(self.cfg, batch["input_ids"], batch["labels"], batch.get("pixel_values"),
                     self.device, stream=stream)

    def manual_training_step(self, batch: Batch, num_items_global: int,
                             last_micro_batch: bool = True) -> torch.Tensor:
        """fwd + bwd of one micro-batch; returns the micro-batch CE SUM (device [1]).
        On the last micro-batch of a step the gradient exchange starts during backward."""
        if self._gate is not None:
            self._gate.region()
        elif getattr(self.opt, "async_update", False):  # ZeRO-2/3: the persistent region
            self.opt.wait_range(0, self._region_end, torch.cuda.current_stream(self.device))
            if self._pending_refresh:
                self.store.refresh_transposed(self._pending_refresh)
            self._pending_refresh = None
        loss_sum = self.engine.forward(batch, 1.0 / max(1, num_items_global))
        if last_micro_batch and self.overlap_comm:
            self.sync.begin_overlap()
        self._offload_final = last_micro_batch
        if self.unit_mode:
            self.sync.final_pass = last_micro_batch
        try:
            self.engine.backward(batch)
        finally:
            self._offload_final = False
            if self.unit_mode:
                self.sync.final_pass = False
        return loss_sum

    def manual_optimization_step(self) -> None:
        self.sync.reduce_grads()
        sumsq = None
        if self.opt.cfg.max_grad_norm and self.opt.cfg.max_grad_norm > 0:
            if self.unit_mode:
                sumsq = self.sync.global_sumsq(K)
            elif self.mode != "ddp":
                sumsq = self.sync.all_reduce_scalar(self.opt.grad_sumsq())
            else:
                sumsq = self.opt.grad_sumsq()
        if self.adam_overlap is not None:
            # update + zero_grad + W^T per unit on the optimizer stream (ddp: no gather)
            self.adam_overlap.step(self.sched.lr(), sumsq)
            self.sched.step()
            return
        # the whole flat gradient is the optimizer's (data parallel): zeroed by the update
        fused_zero = (isinstance(self.opt, FusedAdam) and self.store.grad is not None and
                      self.opt.g.data_ptr() == self.store.grad.data_ptr() and
                      self.opt.g.numel() == self.store.grad.numel())
        if fused_zero:
            self.opt.step(self.sched.lr(), sumsq, zero_grad=True)
        else:
            self.opt.step(self.sched.lr(), sumsq)
        self.sync.gather_params()
        if self._gate is not None:
            self._gate.arm()  # transposes rebuilt per unit once its update has landed
        elif self.unit_mode and getattr(self.opt, "async_update", False):
            # the host update of the persistent region (the tied embedding among it) is
            # still on its way: rebuild its transposes after the region wait at the top of
            # the next micro-step, not now (the transpose would read a half-written E)
            self._pending_refresh = self._refresh
        else:
            self.store.refresh_transposed(self._refresh)
        self.sched.step()
        if not fused_zero:
            self.store.zero_grad()

    def flush(self) -> None:
        """Complete an optimizer update still running on the host (overlapped offload):
        the parameters are final and the compute stream is ordered after their upload."""
        if hasattr(self.opt, "join"):
            self.opt.join()
        if self.adam_overlap is not None:
            self.adam_overlap.join()
        if self._pending_refresh:
            self.store.refresh_transposed(self._pending_refresh)
        self._pending_refresh = None

    def recover(self) -> None:
        """After an exception inside a step (OOM while probing micro-batch sizes): reset
        the engine (activation cache, ZeRO-3 windows), drop the partial gradients and any
        armed overlap, and hand the freed memory back to the device."""
        self.flush()
        self.engine.reset()
        if isinstance(self.sync, GradSync):
            self.sync.reset()
        self.store.zero_grad()
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
            torch.cuda.empty_cache()

    def train_step(self, batches: list[Batch], num_items_global: int) -> torch.Tensor:
        """One optimizer step over `batches` (gradient accumulation)."""
        total = torch.zeros(1, dtype=torch.float32, device=self.device)
        for i, b in enumerate(batches):
            total += self.manual_training_step(b, num_items_global, i == len(batches) - 1)
        self.manual_optimization_step()
        return total


def _fp32_overlap(store, sync, mode) -> int:
    """Length of this rank's optimizer range that lies in the fp32-read region (those
    master values are read by the step on the device and must be copied back)."""
    if mode == "ddp":
        return store.fp32_end
    lo = sync.rank * store.shard_size
    return max(0, min(store.fp32_end - lo, store.shard_size))
