"""Benchmark harness with the reference's API (§8(a) rows a1-a5, a16):
`ManualTrainer` (src/benchmarking/utils.py:40-80), `benchmark_acc_optim_times` /
`estimate_step_time` (src/benchmarking/step_time.py:33-97), `find_max_mbs_pow2`
(src/benchmarking/max_batch_size.py:11-25), `count_flops_per_example`
(src/benchmarking/flops.py:9-37) and `compute_training_days`
(experiments/training_time_empirical.py:133-138).

One deliberate difference: the reference times host wall-clock around calls that
launch asynchronous GPU work and never synchronises ("No device
sync"); `perf_timer` here synchronises the device at both ends, so each time is the
real device time of that phase.  The formula
step_time = mean_acc × (target_mbs // mbs) + mean_optim is unchanged.
"""

from __future__ import annotations

import logging
import time
from contextlib import contextmanager
from types import SimpleNamespace

import torch
import torch.distributed as dist

from . import config as C
from .distributed import sharding_to_mode
from .optim import AdamConfig
from .trainer import ManualTrainer as _StepTrainer
from .trainer import StepConfig

logger = logging.getLogger("academic-pretraining")


def _sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


@contextmanager
def perf_timer():
    """Yields a callable returning the elapsed seconds of the block (device-synced)."""
    _sync()
    t1 = time.perf_counter()
    box = [None]
    yield lambda: box[0]
    _sync()
    box[0] = time.perf_counter() - t1


class ManualTrainer:
    """The reference's ManualTrainer surface over the MI355X step: one object holding
    the model, the data and the fused optimizer/scheduler/exchange.

    manual_training_step(model, inputs): one micro-batch forward + backward with HF
        Trainer loss semantics without num_items_in_batch (mean over the micro-batch's
        label tokens, divided by gradient_accumulation_steps, averaged over DP ranks
        like DDP's gradient averaging);
    manual_optimization_step(model): exchange → clip (max_grad_norm > 0) → Adam(W) →
        lr_scheduler.step → zero_grad.
    """

    def __init__(self, training_class, model, train_dataset, hf_args_overrides: dict):
        tc = training_class
        self.training_class, self.model, self.train_dataset = tc, model, train_dataset
        self.model_wrapped = model
        kw = dict(tc.optimizer_kwargs)
        sched_kw = dict(tc.scheduler_kwargs)
        warm = sched_kw.pop("num_warmup_steps", 0)
        # HF Trainer puts every parameter in a group with args.weight_decay (default 0.0),
        # overriding the optimizer kwarg (effective weight decay 0)
        wd = {**tc.hf_training_args_overrides, **hf_args_overrides}.get("weight_decay", 0.0)
        adam = AdamConfig(lr=kw.get("lr", 1e-3), betas=tuple(kw.get("betas", (0.9, 0.999))),
                          eps=kw.get("eps", 1e-8), weight_decay=wd,
                          adamw=tc.optimizer is torch.optim.AdamW,
                          max_grad_norm=tc.max_grad_norm or 0.0)
        sharding = tc.sharding()
        step_cfg = StepConfig(micro_batch_size=tc.micro_batch_size,
                              grad_accum=tc.gradient_accumulation_steps,
                              sharding=sharding,
                              activation_checkpointing=bool(tc.gradient_checkpointing or
                                                            model.gradient_checkpointing),
                              offload=tc.offload(),
                              scheduler=getattr(tc.scheduler_type, "value", tc.scheduler_type),
                              num_warmup_steps=warm, num_training_steps=tc.num_training_steps,
                              min_lr_rate=sched_kw.get("min_lr_rate", 0.0))
        if sharding_to_mode(sharding) in ("zero2", "zero3") and \
                not model.mmpt_config.freeze_tower_and_llm:
            # ZeRO-2/3 partition the fp32 master, gradients and optimizer state (ZeRO-3 the
            # bf16 weights too): the trainer owns a Zero3Store seeded from the model's
            # initial weights, and the facade's full-size device storage is released
            # (DeepSpeed partitions at init), so the sweep measures the partitioned
            # footprint; gather the weights with core.store.full_master().
            dev = model.store.device
            weights = model.partition_out()
            self.core = _StepTrainer(step_cfg, adam, dev, model_cfg=model.mmpt_config,
                                     store=None, init=False)
            self.core.store.load(weights)
            self.core.store.refresh_shadow()
            del weights
        else:
            self.core = _StepTrainer(step_cfg, adam, model.store.device,
                                     model_cfg=model.mmpt_config, store=model.store,
                                     engine=model.engine)
        self.args = SimpleNamespace(per_device_train_batch_size=tc.micro_batch_size,
                                    gradient_accumulation_steps=tc.gradient_accumulation_steps,
                                    max_grad_norm=tc.max_grad_norm)
        self._epoch = 0
        self._micro = 0  # micro-batches since the last optimizer step

    @classmethod
    def from_trainer(cls, trainer: "ManualTrainer") -> "ManualTrainer":
        """Reference: prepares an HF Trainer for manual stepping.  The MI355X trainer
        is built ready; kept so reference call sites read unchanged."""
        return trainer

    # ---------------------------------------------------------------- data
    def get_train_dataloader(self, micro_batch_size: int | None = None):
        """Infinite iterator of collated micro-batches; each DP rank reads a disjoint,
        rank-strided slice of a per-epoch permutation (DistributedSampler order)."""
        mbs = micro_batch_size or self.args.per_device_train_batch_size
        ds = self.train_dataset
        world, rank = self.core.world, self.core.rank
        while True:
            g = torch.Generator().manual_seed(1234 + self._epoch)
            order = torch.randperm(len(ds), generator=g)[rank::world].tolist()
            self._epoch += 1
            for i in range(0, len(order) - mbs + 1, mbs):
                items = [ds[j] for j in order[i:i + mbs]]
                yield {k: torch.stack([it[k] for it in items]) for k in items[0]}

    # ---------------------------------------------------------------- steps
    def manual_training_step(self, model, inputs: dict) -> torch.Tensor:
        b = self.core.stage(inputs)
        denom = max(1, b.num_items) * self.args.gradient_accumulation_steps * self.core.world
        self._micro += 1
        # like accelerator.accumulate: the gradient exchange starts only on the last
        # micro-batch of the accumulation window
        last = self._micro % self.args.gradient_accumulation_steps == 0
        loss_sum = self.core.manual_training_step(b, denom, last_micro_batch=last)
        return loss_sum.detach() / max(1, b.num_items)

    def manual_optimization_step(self, model) -> None:
        self.core.manual_optimization_step()
        # the optimizer time the harness reports includes the whole update (an overlapped
        # host update would otherwise be charged to the next accumulation step)
        self.core.flush()
        self._micro = 0

    def recover(self) -> None:
        """Clean state after an OOM inside a step (trainer.ManualTrainer.recover)."""
        self.core.recover()
        self._micro = 0


def benchmark_acc_optim_times(trainer: ManualTrainer, micro_batch_size: int, training_steps: int = 1,
                              accumulations: int = 1, warmup: bool = False) -> tuple[float, float]:
    """step_time.py:33-72: `training_steps` × (`accumulations` micro-steps + one optimizer
    step); with warmup, one extra leading step is run and discarded."""
    torch.cuda.empty_cache()
    acc, opt = [], []
    steps = training_steps + (1 if warmup else 0)
    model = trainer.model_wrapped
    data = trainer.get_train_dataloader(micro_batch_size)
    for _ in range(steps):
        for _ in range(accumulations):
            inputs = next(data)
            with perf_timer() as t:
                trainer.manual_training_step(model, inputs)
            acc.append(t())
        with perf_timer() as t:
            trainer.manual_optimization_step(model)
        opt.append(t())
    if warmup:  # the reference drops exactly one entry of each list
        acc, opt = acc[1:], opt[1:]
    logger.info("Accumulation times: %s", acc)
    logger.info("Optimization times: %s", opt)
    return sum(acc) / len(acc), sum(opt) / len(opt)


def estimate_step_time(trainer: ManualTrainer, micro_batch_size: int, target_micro_batch_size: int,
                       num_benchmarking_steps: int) -> float:
    """step_time.py:75-97: mean_acc × (target_mbs // mbs) + mean_optim."""
    accumulation_steps = target_micro_batch_size // micro_batch_size
    mean_acc, mean_opt = benchmark_acc_optim_times(trainer, micro_batch_size,
                                                   training_steps=num_benchmarking_steps,
                                                   accumulations=1, warmup=True)
    return mean_acc * accumulation_steps + mean_opt


def find_max_mbs_pow2(trainer: ManualTrainer, limit: int) -> int:
    """max_batch_size.py:11-25: largest power of two ≤ limit whose step does not OOM."""
    mbs = 1
    while mbs <= limit:
        try:
            benchmark_acc_optim_times(trainer, micro_batch_size=mbs, training_steps=1, accumulations=1)
        except torch.cuda.OutOfMemoryError:
            trainer.recover()  # the failed micro-batch's cache / windows must not survive
            break
        mbs *= 2
    return mbs // 2


def count_flops_per_example(model_class) -> float:
    """flops.py:9-37 counts one fwd+bwd of a batch-1 sample with FlopCounterMode on the
    eager model (full-square attention).  Restated analytically (config.flops_per_sample):
    3 × forward matmul FLOPs at the model class's sequence length."""
    cfg = model_class.model_config
    n_img = cfg.vision.num_patches if cfg.vision is not None else 0
    return C.flops_per_sample(cfg, model_class.sequence_length - n_img)


def compute_training_days(step_time: float | None, num_steps: int) -> float | None:
    """training_time_empirical.py:133-138 (takes the step time directly)."""
    if step_time is None:
        return None
    return num_steps * step_time / (24 * 60 * 60)


def all_ranks_max(x: float) -> float:
    """Max of a host float over the DP ranks (the slowest rank sets the step time)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return x
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
