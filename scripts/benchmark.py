#!/usr/bin/env python
"""Drop-in for the reference's `scripts/benchmark.py` (scripts/benchmark.py:13-79): the
empirical training-time sweep over the method space for one (nodes, GPUs, GPU type,
model), on MI355X through this package.

    python scripts/benchmark.py --num-nodes 1 --gpus-per-node 8 --gpu-type mi355x \
        --model vit-b16-pythia-1b --methods all --cmd run

Same flags and semantics (argparse instead of tyro, which is not installed):
methods naive → one config; free-lunch → free_lunch=True; all → free_lunch × activation
checkpointing × {"", zero_1, zero_2, zero_3, fsdp_shard_grad_op, fsdp_full_shard} ×
offloading, invalid combinations dropped (TrainingTimeEmpirical.is_valid).
cmd: run | count | print-incomplete | print-results.  Results: $MMPT_RESULTS_DIR.
"""

import argparse
import math
import os
import signal
import sys
from typing import get_args

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from multimodal_llm_pretraining_amd.gpus import GPUS, ampere_or_newer_gpu  # noqa: E402
from multimodal_llm_pretraining_amd.models import ModelT, get_model_class  # noqa: E402
from multimodal_llm_pretraining_amd.sweep import TrainingTimeEmpiricalSweep  # noqa: E402


def model_types() -> list[str]:
    out = []
    for part in get_args(ModelT):  # Literal of Literals flattens on Python ≥ 3.9.1
        out += list(get_args(part)) if get_args(part) else [part]
    return out


def validate_arguments(num_nodes: int, gpus_per_node: int, gpu_type: str, model: str) -> None:
    model_class = get_model_class(model)
    num_gpus = num_nodes * gpus_per_node
    assert model_class.batch_size % num_gpus == 0, (
        f"model batch size ({model_class.batch_size}) should be evenly divisible by total GPUs ({num_gpus})")
    assert math.log2(model_class.batch_size // num_gpus).is_integer(), (
        f"batch size per gpu ({model_class.batch_size // num_gpus}) should be power of 2")
    if model_class.mixed_precision == "bf16":
        assert ampere_or_newer_gpu(gpu_type), "GPU must be ampere or newer to use mixed precision with bf16"


def search_space(num_nodes, gpus_per_node, gpu_type, model, methods) -> dict:
    free_lunch, ac, sharding, offloading = [False], [False], [""], [False]
    if methods == "free-lunch":
        free_lunch = [True]
    elif methods == "all":
        free_lunch = [True]
        ac = [False, True]
        sharding = ["", "zero_1", "zero_2", "zero_3", "fsdp_shard_grad_op", "fsdp_full_shard"]
        offloading = [False, True]
    return dict(num_nodes=[num_nodes], gpus_per_node=[gpus_per_node], gpu_type=[gpu_type],
                model=[model], free_lunch=free_lunch, activation_checkpointing=ac,
                sharding=sharding, offloading=offloading)


def run_benchmark(num_nodes, gpus_per_node, gpu_type, model, methods="all", cmd="run",
                  slurm=False) -> None:
    validate_arguments(num_nodes, gpus_per_node, gpu_type, model)
    sweep = TrainingTimeEmpiricalSweep(search_space(num_nodes, gpus_per_node, gpu_type, model,
                                                    methods))
    TrainingTimeEmpiricalSweep.run(experiment_sweep=sweep, cmd=cmd, slurm=slurm)


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description="empirical training-time sweep (MI355X)")
    ap.add_argument("--num-nodes", type=int, required=True)
    ap.add_argument("--gpus-per-node", type=int, required=True)
    ap.add_argument("--gpu-type", required=True, choices=GPUS)
    ap.add_argument("--model", required=True, choices=model_types())
    ap.add_argument("--methods", default="all", choices=["naive", "free-lunch", "all"])
    ap.add_argument("--cmd", default="run",
                    choices=["run", "count", "print-incomplete", "print-results"])
    ap.add_argument("--slurm", action="store_true")
    a = ap.parse_args(argv)
    run_benchmark(a.num_nodes, a.gpus_per_node, a.gpu_type, a.model, a.methods, a.cmd, a.slurm)


if __name__ == "__main__":
    try:
        main()
    except KeyboardInterrupt:
        sys.exit(128 + signal.SIGINT)
