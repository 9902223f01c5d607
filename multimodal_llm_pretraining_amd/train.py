"""TrainingClass (§8(a) row a6): the reference's knob set → HF TrainingArguments
dict / DeepSpeed config / FSDP options (src/train.py:16-215), and `build_trainer`,
which here returns the MI355X manual trainer (benchmarking.ManualTrainer) instead of
a transformers.Trainer.

`_to_huggingface_args_dict`, `_build_deepspeed_config` and `_build_fsdp_config`
produce the same dict as the reference for the same knobs (pinned by the JSON in the
reference README, tests/golden/training_arguments_readme.json), including its quirk
that `num_warmup_steps` is popped out of `scheduler_kwargs` on every call.

Which knobs the MI355X step executes (everything else raises in build_trainer):
  precision bf16 (a14); optimizer Adam/AdamW (fused HIP Adam); schedulers of
  optim.Schedule; max_grad_norm; DDP, ZeRO-1/2/3 (+ FSDP shard_grad_op = ZeRO-2,
  full_shard / hybrid_shard on one node = ZeRO-3), optimizer offload to the host,
  gradient_checkpointing (per-layer recompute).  tf32/compile are accepted and have no
  effect (no tracing compiler; every GEMM is bf16 MFMA); ZeRO-3++'s quantized
  collectives run as exact ZeRO-3.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Literal

import torch

FsdpShardingT = Literal["no_shard", "shard_grad_op", "full_shard", "hybrid_shard_zero2", "hybrid_shard"]
ZeroStageT = Literal["0", "1", "2", "3", "3++"]


def _sched_value(s) -> str:
    return getattr(s, "value", s)


@dataclass
class TrainingClass:
    num_training_steps: int
    micro_batch_size: int
    gradient_accumulation_steps: int
    gradient_checkpointing: bool = False
    bf16: bool = False
    fp16: bool = False
    tf32: bool = False
    compile: bool = False

    optimizer: type = torch.optim.AdamW
    optimizer_kwargs: dict[str, Any] = field(default_factory=dict)
    scheduler_type: Any = "linear"
    scheduler_kwargs: dict[str, Any] = field(default_factory=dict)

    FsdpShardingT = FsdpShardingT
    fsdp_sharding: str = "no_shard"
    fsdp_layers_to_wrap: list[str] = field(default_factory=list)
    fsdp_offload: bool = False

    ZeroStageT = ZeroStageT
    zero_stage: str = "0"
    zero_offload_optimizer: bool = False
    zero_offload_params: bool = False

    max_grad_norm: float = 1.0
    hf_training_args_overrides: dict[str, Any] = field(default_factory=dict)

    # ------------------------------------------------------------ validity (train.py:42-52)
    def is_valid(self) -> bool:
        bad = (
            self.num_training_steps <= 0,
            self.micro_batch_size <= 0,
            self.gradient_accumulation_steps <= 0,
            self.bf16 and self.fp16,
            self.fsdp_sharding != "no_shard" and self.zero_stage != "0",
            self.fsdp_offload and self.fsdp_sharding == "no_shard",
            self.zero_offload_optimizer and self.zero_stage == "0",
            self.zero_offload_params and self.zero_stage not in ("3", "3++"),
        )
        return not any(bad)

    # ------------------------------------------------------------ HF arguments
    def to_huggingface_args(self, **hf_training_args_overrides):
        from transformers import TrainingArguments

        return TrainingArguments(**self._to_huggingface_args_dict(**hf_training_args_overrides))

    def _to_huggingface_args_dict(self, **hf_training_args_overrides) -> dict:
        fsdp_options, fsdp_config = self._build_fsdp_config()
        ds_config = self._build_deepspeed_config()
        warmup = self.scheduler_kwargs.pop("num_warmup_steps", 0)  # reference pops (mutates)
        out = {
            "max_steps": self.num_training_steps,
            "per_device_train_batch_size": self.micro_batch_size,
            "gradient_accumulation_steps": self.gradient_accumulation_steps,
            "lr_scheduler_type": _sched_value(self.scheduler_type),
            "lr_scheduler_kwargs": self.scheduler_kwargs,
            "warmup_steps": warmup,
            "gradient_checkpointing": self.gradient_checkpointing,
            "bf16": self.bf16,
            "fp16": self.fp16,
            "tf32": self.tf32,
            "fsdp": fsdp_options,
            "fsdp_config": fsdp_config,
            "deepspeed": ds_config,
            "ddp_find_unused_parameters": False,
            "torch_compile": self.compile,
            "max_grad_norm": self.max_grad_norm,
        }
        for extra in (self.hf_training_args_overrides, hf_training_args_overrides):
            dup = set(extra) & set(out)
            if dup:  # the reference builds dict(..., **a, **b): a repeated key is a TypeError
                raise TypeError(f"got multiple values for keyword argument {sorted(dup)[0]!r}")
            out.update(extra)
        return out

    def _build_fsdp_config(self):
        if self.fsdp_sharding == "no_shard":
            return "", None
        opts = [self.fsdp_sharding, "auto_wrap"] + (["offload"] if self.fsdp_offload else [])
        return opts, {"transformer_layer_cls_to_wrap": self.fsdp_layers_to_wrap}

    def _build_deepspeed_config(self) -> dict | None:
        if self.zero_stage == "0":
            return None
        cfg: dict[str, Any] = {
            "fp16": {"enabled": "auto", "loss_scale": 0, "loss_scale_window": 1000,
                     "initial_scale_power": 16, "hysteresis": 2, "min_loss_scale": 1},
            "gradient_accumulation_steps": "auto",
            "gradient_clipping": "auto",
            "train_batch_size": "auto",
            "train_micro_batch_size_per_gpu": "auto",
        }
        if self.optimizer in (torch.optim.Adam, torch.optim.AdamW):
            cfg["optimizer"] = {"type": "Adam", "params": {
                "lr": "auto", "betas": "auto", "eps": "auto", "weight_decay": "auto",
                "adam_w_mode": self.optimizer is torch.optim.AdamW}}
        if self.zero_stage == "1":
            cfg["zero_optimization"] = {"stage": 1}
        elif self.zero_stage == "2":
            cfg["zero_optimization"] = {
                "stage": 2, "allgather_partitions": True, "allgather_bucket_size": 2e8,
                "overlap_comm": True, "reduce_scatter": True, "reduce_bucket_size": 2e8,
                "contiguous_gradients": True}
        elif self.zero_stage in ("3", "3++"):
            z = {"stage": 3, "overlap_comm": True, "contiguous_gradients": True,
                 "sub_group_size": 1e9, "reduce_bucket_size": "auto",
                 "stage3_prefetch_bucket_size": "auto",
                 "stage3_param_persistence_threshold": "auto",
                 "stage3_max_live_parameters": 1e9, "stage3_max_reuse_distance": 1e9,
                 "stage3_gather_16bit_weights_on_model_save": True}
            if self.zero_stage == "3++":
                z.update(zero_quantized_weights=True,
                         zero_hpz_partition_size=torch.cuda.device_count(),
                         zero_quantized_gradients=True)
            cfg["zero_optimization"] = z
        if self.zero_offload_optimizer:
            cfg["zero_optimization"]["offload_optimizer"] = {"device": "cpu", "pin_memory": True}
        if self.zero_offload_params:
            cfg["zero_optimization"]["offload_param"] = {"device": "cpu", "pin_memory": True}
        return cfg

    # ------------------------------------------------------------ MI355X execution
    def sharding(self) -> str:
        """The exchange mode the MI355X step runs for these knobs (distributed.py,
        zero3.py)."""
        if self.fsdp_sharding != "no_shard":
            return {"shard_grad_op": "fsdp_shard_grad_op", "full_shard": "fsdp_full_shard",
                    "hybrid_shard_zero2": "fsdp_hybrid_shard_zero2",
                    "hybrid_shard": "fsdp_hybrid_shard"}[self.fsdp_sharding]
        return {"0": "", "1": "zero_1", "2": "zero_2", "3": "zero_3", "3++": "zero_3++"}[self.zero_stage]

    def offload(self) -> bool:
        """Optimizer state (and, for ZeRO-3/FSDP, DeepSpeed's parameter offload) → host
        memory.  The MI355X step offloads the fp32 master + Adam state and runs the
        update on the host (offload.HostAdam); the bf16 parameters the step reads stay
        in HBM (288 GB holds every model of the sweep)."""
        return bool(self.fsdp_offload or self.zero_offload_optimizer or self.zero_offload_params)

    def build_trainer(self, model, train_dataset, hf_training_args_overrides: dict | None = None,
                      hf_trainer_kwargs_overrides: dict | None = None):
        """→ benchmarking.ManualTrainer driving `model` (an MMPTForPretraining)."""
        from .benchmarking import ManualTrainer

        if not self.is_valid():
            raise ValueError("invalid TrainingClass knob combination")
        if not self.bf16 or self.fp16:
            raise NotImplementedError("the MI355X step computes in bf16 autocast semantics; "
                                      "set bf16=True (fp16/fp32 recipes are not on the path)")
        if self.optimizer not in (torch.optim.Adam, torch.optim.AdamW):
            raise NotImplementedError(f"optimizer {self.optimizer!r}: only Adam/AdamW are fused")
        return ManualTrainer(self, model, train_dataset, dict(hf_training_args_overrides or {}))
