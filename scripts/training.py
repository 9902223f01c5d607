#!/usr/bin/env python
"""Drop-in for the reference's `scripts/training.py` (:15-130): train a model type from a
TrainingArguments JSON (the file `scripts/to_training_arguments.py` writes) — here on the
MI355X step instead of a transformers.Trainer over DeepSpeed/FSDP.

    python scripts/training.py --output-dir out --model-type vit-b16-pythia-1b \
        --training-arguments args.json [--max-steps 10]
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        scripts/training.py ...          # one process per GPU (torchrunx is not installed)

TrainingArguments keys honoured (everything the reference's JSON sets):
  per_device_train_batch_size, gradient_accumulation_steps, max_steps, lr_scheduler_type,
  lr_scheduler_kwargs.min_lr_rate, warmup_steps, gradient_checkpointing, bf16 (must be
  true: the step computes in bf16 autocast semantics), max_grad_norm, seed, and the
  sharding given by `deepspeed.zero_optimization` (stage, offload_optimizer,
  offload_param) or `fsdp` ("shard_grad_op" / "full_shard" / "hybrid_shard[_zero2]"
  + "offload").  tf32 / torch_compile / fsdp_config are accepted and have no effect.
Optimizer: the model class's (Adam/AdamW + its kwargs) — or, when a DeepSpeed config is
given, its optimizer block with "auto" values resolved to the TrainingArguments defaults
(learning_rate 5e-5, adam_beta1/2 0.9/0.999, adam_epsilon 1e-8, weight_decay 0), as HF's
DeepSpeed integration does.  Weight decay is the TrainingArguments value
(default 0) in both cases, as HF's parameter groups apply it.
Data: the model class's dummy dataset (the reference has no dataset for these model types
either); --data-path / --data-split are accepted for CLI compatibility.
Writes one JSON line per optimizer step to <output-dir>/trainer_log.jsonl.

CPU (BASELINE C1, `--methods naive` plumbing on a host without a GPU, or --cpu): the
model class's `build_model(use_custom_kernels=False)` — the plain transformers model, eager
attention, fp32 (fp16/bf16 mixed precision is a GPU setting; the CPU run is fp32 as the
reference's CPU Trainer runs it) — trained with the model class's torch optimizer, the
TrainingArguments schedule and max_grad_norm, world size 1 (scripts/training.py:73-104 of
the reference, without torchrunx).  Never a fallback for the GPU step: it is chosen only
when no GPU is visible or --cpu is given.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def sharding_from_args(args: dict) -> tuple[str, bool]:
    """(sharding string of experiments/config.py, offload?) from a TrainingArguments dict."""
    ds = args.get("deepspeed")
    if isinstance(ds, str) and ds:
        with open(ds) as f:
            ds = json.load(f)
    if ds:
        z = ds.get("zero_optimization", {}) or {}
        stage = str(z.get("stage", 0))
        if z.get("zero_quantized_weights") or z.get("zero_quantized_gradients"):
            stage = "3++"
        off = bool(z.get("offload_optimizer") or z.get("offload_param"))
        return ({"0": "", "1": "zero_1", "2": "zero_2", "3": "zero_3", "3++": "zero_3++"}[stage], off)
    fsdp = args.get("fsdp") or ""
    opts = fsdp.split() if isinstance(fsdp, str) else list(fsdp)
    for mode in ("shard_grad_op", "full_shard", "hybrid_shard_zero2", "hybrid_shard"):
        if mode in opts:
            return "fsdp_" + mode, "offload" in opts
    return "", False


def adam_from_args(args: dict, model_class):
    import torch

    from multimodal_llm_pretraining_amd.optim import AdamConfig

    wd = float(args.get("weight_decay", 0.0))
    clip = float(args.get("max_grad_norm", 1.0) or 0.0)
    ds = args.get("deepspeed")
    if isinstance(ds, dict) and ds.get("optimizer"):
        p = ds["optimizer"].get("params", {})

        def auto(key, default):
            v = p.get(key, "auto")
            return default if v == "auto" else v

        betas = auto("betas", (args.get("adam_beta1", 0.9), args.get("adam_beta2", 0.999)))
        return AdamConfig(lr=float(auto("lr", args.get("learning_rate", 5e-5))),
                          betas=tuple(betas), eps=float(auto("eps", args.get("adam_epsilon", 1e-8))),
                          weight_decay=float(auto("weight_decay", wd)),
                          adamw=bool(p.get("adam_w_mode", True)), max_grad_norm=clip)
    kw = dict(model_class.optimizer_kwargs)
    return AdamConfig(lr=kw.get("lr", 1e-3), betas=tuple(kw.get("betas", (0.9, 0.999))),
                      eps=kw.get("eps", 1e-8), weight_decay=wd,
                      adamw=model_class.optimizer is torch.optim.AdamW, max_grad_norm=clip)


def _log(output_dir: str, rec: dict) -> None:
    print(json.dumps(rec), flush=True)
    with open(os.path.join(output_dir, "trainer_log.jsonl"), "a") as f:
        f.write(json.dumps(rec) + "\n")


def train_cpu(output_dir: str, model_type: str, training_arguments: dict,
              max_steps: int | None = None, log_every: int = 1) -> list[dict]:
    """BASELINE C1: the naive eager model on the CPU, world size 1, fp32."""
    import torch

    from multimodal_llm_pretraining_amd.models import get_model_class
    from multimodal_llm_pretraining_amd.optim import Schedule

    a = training_arguments
    if int(os.environ.get("WORLD_SIZE", "1")) != 1:
        raise NotImplementedError("the CPU path runs at world size 1 (BASELINE C1)")
    mc = get_model_class(model_type)
    torch.manual_seed(int(a.get("seed", 42)))
    model = mc.build_model(use_custom_kernels=False)
    if a.get("gradient_checkpointing", False):
        model.gradient_checkpointing_enable()
    model.train()
    kw = dict(mc.optimizer_kwargs)
    # HF's parameter groups apply TrainingArguments.weight_decay (default 0)
    kw["weight_decay"] = float(a.get("weight_decay", 0.0))
    opt = mc.optimizer(model.parameters(), **kw)
    mbs = int(a.get("per_device_train_batch_size", 8))
    ga = int(a.get("gradient_accumulation_steps", 1))
    steps = int(max_steps if max_steps is not None else a.get("max_steps", mc.training_steps))
    sched_kw = a.get("lr_scheduler_kwargs") or {}
    sched = Schedule(kw["lr"], str(a.get("lr_scheduler_type", "linear")),
                     int(a.get("warmup_steps", 0)), int(a.get("max_steps", steps)),
                     float(sched_kw.get("min_lr_rate", 0.0)))
    clip = float(a.get("max_grad_norm", 1.0) or 0.0)
    ds = mc.load_dummy_dataset()
    os.makedirs(output_dir, exist_ok=True)
    log, cursor = [], 0
    for step in range(steps):
        t0 = time.perf_counter()
        micro = []
        for _ in range(ga):
            items = [ds[(cursor + i) % len(ds)] for i in range(mbs)]
            micro.append({k: torch.stack([it[k] for it in items]) for k in items[0]})
            cursor += mbs
        # HF Trainer: loss = CE sum / label tokens of the whole accumulation window
        n_items = sum(int((b["labels"][:, 1:] != -100).sum()) for b in micro)
        lr = sched.lr()
        for gr in opt.param_groups:
            gr["lr"] = lr
        total = 0.0
        for b in micro:
            loss = model(**b, num_items_in_batch=n_items).loss
            loss.backward()
            total += loss.item()
        if clip > 0:
            torch.nn.utils.clip_grad_norm_(model.parameters(), clip)
        opt.step()
        sched.step()
        opt.zero_grad(set_to_none=True)
        rec = {"step": step + 1, "loss": total, "learning_rate": lr,
               "step_time_s": round(time.perf_counter() - t0, 4), "samples": mbs * ga,
               "device": "cpu", "precision": "fp32"}
        log.append(rec)
        if (step + 1) % log_every == 0:
            _log(output_dir, rec)
    return log


def train(output_dir: str, model_type: str, training_arguments: dict, max_steps: int | None = None,
          log_every: int = 1, cpu: bool = False) -> list[dict]:
    import torch
    import torch.distributed as dist

    if cpu or not torch.cuda.is_available():
        return train_cpu(output_dir, model_type, training_arguments, max_steps, log_every)

    from multimodal_llm_pretraining_amd.models import get_model_class
    from multimodal_llm_pretraining_amd.trainer import ManualTrainer, StepConfig

    a = training_arguments
    if not a.get("bf16", False) or a.get("fp16", False):
        raise NotImplementedError("the MI355X step computes in bf16 autocast semantics (bf16=true)")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1 and not dist.is_initialized():
        dist.init_process_group("nccl", device_id=device)
    mc = get_model_class(model_type)
    sharding, offload = sharding_from_args(a)
    mbs = int(a.get("per_device_train_batch_size", 8))
    ga = int(a.get("gradient_accumulation_steps", 1))
    steps = int(max_steps if max_steps is not None else a.get("max_steps", mc.training_steps))
    sched_kw = a.get("lr_scheduler_kwargs") or {}
    tr = ManualTrainer(
        StepConfig(model=model_type, micro_batch_size=mbs, grad_accum=ga, sharding=sharding,
                   activation_checkpointing=bool(a.get("gradient_checkpointing", False)),
                   offload=offload, seed=int(a.get("seed", 42)),
                   scheduler=str(a.get("lr_scheduler_type", "linear")),
                   num_warmup_steps=int(a.get("warmup_steps", 0)),
                   num_training_steps=int(a.get("max_steps", steps)),
                   min_lr_rate=float(sched_kw.get("min_lr_rate", 0.0))),
        adam_from_args(a, mc), device)
    ds = mc.load_dummy_dataset()
    os.makedirs(output_dir, exist_ok=True)
    log = []
    cursor = 0
    for step in range(steps):
        t0 = time.perf_counter()
        batches = []
        for _ in range(ga):
            # rank-strided slice of the per-step global batch (DistributedSampler order)
            idx = [(cursor + (i * world + rank)) % len(ds) for i in range(mbs)]
            items = [ds[j] for j in idx]
            batches.append(tr.stage({k: torch.stack([it[k] for it in items]) for k in items[0]}))
            cursor += mbs * world
        n = torch.tensor([sum(b.num_items for b in batches)], dtype=torch.float64, device=device)
        if world > 1:
            dist.all_reduce(n)
        n_items = int(n.item())
        lr = tr.sched.lr()
        loss = tr.train_step(batches, n_items)
        if world > 1:
            dist.all_reduce(loss)
        torch.cuda.synchronize()
        rec = {"step": step + 1, "loss": loss.item() / n_items, "learning_rate": lr,
               "step_time_s": round(time.perf_counter() - t0, 4),
               "samples": mbs * ga * world}
        log.append(rec)
        if rank == 0 and (step + 1) % log_every == 0:
            _log(output_dir, rec)
    if hasattr(tr, "flush"):
        tr.flush()  # an overlapped host optimizer update of the last step
    if world > 1:
        dist.destroy_process_group()
    return log


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description="train a model type from a TrainingArguments JSON")
    ap.add_argument("--output-dir", required=True)
    ap.add_argument("--model-type", required=True)
    ap.add_argument("--training-arguments", required=True, help="path to the JSON")
    ap.add_argument("--data-path", default=None)
    ap.add_argument("--data-split", default=None)
    ap.add_argument("--max-steps", type=int, default=None, help="override max_steps")
    ap.add_argument("--cpu", action="store_true",
                    help="run the naive eager model on the CPU (BASELINE C1); implied without a GPU")
    a = ap.parse_args(argv)
    with open(a.training_arguments) as f:
        targs = json.load(f)
    targs = targs.get("args", targs)
    if a.data_path:
        print("note: --data-path ignored; training on the model class's dummy dataset", flush=True)
    train(a.output_dir, a.model_type, targs, a.max_steps, cpu=a.cpu)


if __name__ == "__main__":
    main()
