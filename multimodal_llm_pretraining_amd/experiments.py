"""Experiment configuration (§8(a) row a7 and the driver of a3-a5):
`TrainingConfig.training_class` (experiments/config.py:38-101) and the
empirical training-time experiment (experiments/training_time_empirical.py:17-238)
without the reference's tango cache / torchrunx launcher: one process per GPU is
started by torch.distributed.run, and `TrainingTimeEmpirical.run()` executes the
three steps (largest micro-batch, step time, training days) in that process group.
"""

from __future__ import annotations

import dataclasses
import math
from dataclasses import dataclass

import torch
import torch.distributed as dist

from .benchmarking import (all_ranks_max, compute_training_days, estimate_step_time,
                           find_max_mbs_pow2)
from .gpus import ampere_or_newer_gpu, tf32_capable
from .models import get_model_class
from .train import TrainingClass

SHARDINGS = ("", "fsdp_shard_grad_op", "fsdp_full_shard", "fsdp_hybrid_shard_zero2",
             "fsdp_hybrid_shard", "zero_1", "zero_2", "zero_3", "zero_3++")


@dataclass
class TrainingConfig:
    num_nodes: int
    gpus_per_node: int
    gpu_type: str
    model: str
    free_lunch: bool = False
    activation_checkpointing: bool = False
    sharding: str = ""
    offloading: bool = False

    def __post_init__(self):
        if self.sharding not in SHARDINGS:
            raise ValueError(f"sharding {self.sharding!r} not in {SHARDINGS}")

    def ampere_or_newer_gpu(self) -> bool:
        return ampere_or_newer_gpu(self.gpu_type)

    def model_class(self):
        return get_model_class(self.model)

    def training_class(self, **training_class_overrides) -> TrainingClass:
        mc = self.model_class()
        fsdp_sharding, fsdp_layers, fsdp_offload = "no_shard", [], False
        zero_stage, zero_off_opt, zero_off_params = "0", False, False
        if self.sharding.startswith("fsdp_"):
            fsdp_sharding = self.sharding[len("fsdp_"):]
            fsdp_layers = mc.fsdp_layers_to_wrap
            fsdp_offload = self.offloading
        elif self.sharding.startswith("zero_"):
            zero_stage = self.sharding[len("zero_"):]
            zero_off_opt = self.offloading
            zero_off_params = self.offloading and zero_stage in ("3", "3++")
        tc = TrainingClass(
            num_training_steps=mc.training_steps,
            micro_batch_size=1,
            gradient_accumulation_steps=1,
            gradient_checkpointing=self.activation_checkpointing,
            bf16=mc.mixed_precision == "bf16",
            fp16=mc.mixed_precision == "fp16",
            tf32=self.free_lunch and tf32_capable(self.gpu_type),
            compile=self.free_lunch and mc.supports_compilation,
            optimizer=mc.optimizer,
            optimizer_kwargs=mc.optimizer_kwargs,
            scheduler_type=mc.scheduler_type,
            scheduler_kwargs=mc.scheduler_kwargs,
            fsdp_sharding=fsdp_sharding,
            fsdp_layers_to_wrap=fsdp_layers,
            fsdp_offload=fsdp_offload,
            zero_stage=zero_stage,
            zero_offload_optimizer=zero_off_opt,
            zero_offload_params=zero_off_params,
            max_grad_norm=mc.max_grad_norm,
            hf_training_args_overrides=mc.hf_training_args,
        )
        return dataclasses.replace(tc, **training_class_overrides)


def build_benchmarking_trainer(config: TrainingConfig, num_samples: int | None = None):
    """training_time_empirical.py:17-40: a 1-step, mbs-1, GA-1 trainer over the model
    class's dummy dataset (compile knobs have no effect on this path)."""
    tc = config.training_class(num_training_steps=1, micro_batch_size=1,
                               gradient_accumulation_steps=1)
    mc = config.model_class()
    model = mc.build_model(use_custom_kernels=True)
    ds = mc.load_dummy_dataset() if num_samples is None else mc.load_dummy_dataset(num_samples=num_samples)
    return tc.build_trainer(model=model, train_dataset=ds)


@dataclass
class TrainingTimeEmpirical:
    config: TrainingConfig
    benchmarking_steps: int = 3
    trial: int = 0

    def __post_init__(self):
        self.model_class = self.config.model_class()
        self.training_class = self.config.training_class()

    @property
    def world(self) -> int:
        return self.config.num_nodes * self.config.gpus_per_node

    def is_valid(self) -> bool:
        """training_time_empirical.py:168-189."""
        bs, n = self.model_class.batch_size, self.world
        per_gpu = bs // n
        bad = (
            self.benchmarking_steps <= 0,
            self.trial < 0,
            bs % n > 0,
            per_gpu <= 0 or not math.log2(per_gpu).is_integer(),
            self.config.activation_checkpointing and not self.model_class.supports_activation_checkpointing,
            self.model_class.mixed_precision == "bf16" and not self.config.ampere_or_newer_gpu(),
            self.config.num_nodes == 1 and self.config.gpus_per_node == 1
            and self.config.sharding != "" and not self.config.offloading,
            self.config.offloading and self.config.sharding == "",
        )
        return not any(bad) and self.training_class.is_valid()

    @property
    def target_micro_batch_size(self) -> int:
        return self.model_class.batch_size // self.world

    def run(self, max_micro_batch_size: int | None = None, num_samples: int | None = None) -> dict:
        """largest power-of-two micro-batch → step time (halving on OOM) → training days."""
        if dist.is_initialized() and dist.get_world_size() != self.world:
            raise ValueError("process group size differs from num_nodes × gpus_per_node")
        trainer = build_benchmarking_trainer(self.config, num_samples)
        max_mbs = max_micro_batch_size or find_max_mbs_pow2(trainer, limit=self.target_micro_batch_size)
        mbs, result = max_mbs, None
        while mbs > 0:
            try:
                st = estimate_step_time(trainer, mbs, self.target_micro_batch_size,
                                        self.benchmarking_steps)
                result = {"micro_batch_size": mbs, "step_time": all_ranks_max(st),
                          "compile_disabled": True}
                break
            except torch.cuda.OutOfMemoryError:
                trainer.recover()
                mbs //= 2
        return {"max_micro_batch_size": max_mbs, **(result or {}),
                "training_days": compute_training_days(result and result["step_time"],
                                                       self.model_class.training_steps)}
