#!/usr/bin/env python
"""Drop-in for the reference's `scripts/print_optimal_config.py` (:8-48): read the cached
sweep results for one (nodes, GPUs, GPU type, model) over the full method space and print
them sorted by training_days (fastest first), with grad_acc_steps =
batch_size // (micro_batch_size × gpus_per_node) as the reference computes it.

    python scripts/print_optimal_config.py --num-nodes 1 --gpus-per-node 8 \
        --gpu-type mi355x --model vit-b16-pythia-1b
"""

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from benchmark import model_types  # noqa: E402

from multimodal_llm_pretraining_amd.gpus import GPUS  # noqa: E402
from multimodal_llm_pretraining_amd.models import get_model_class  # noqa: E402
from multimodal_llm_pretraining_amd.sweep import TrainingTimeEmpiricalSweep, print_table  # noqa: E402

COLUMNS = ["num_nodes", "gpus_per_node", "gpu_type", "model", "free_lunch",
           "activation_checkpointing", "sharding", "offloading", "micro_batch_size",
           "grad_acc_steps", "training_days"]


def optimal_configs(num_nodes, gpus_per_node, gpu_type, model) -> list[dict]:
    rows = TrainingTimeEmpiricalSweep(dict(
        num_nodes=[num_nodes], gpus_per_node=[gpus_per_node], gpu_type=[gpu_type], model=[model],
        free_lunch=[False, True], activation_checkpointing=[False, True],
        sharding=["", "zero_1", "zero_2", "zero_3", "fsdp_shard_grad_op", "fsdp_full_shard"],
        offloading=[False, True])).results()
    batch_size = get_model_class(model).batch_size
    rows = sorted((r for r in rows if r.get("training_days") is not None),
                  key=lambda r: r["training_days"])
    for r in rows:
        r["grad_acc_steps"] = batch_size // (r["micro_batch_size"] * r["gpus_per_node"])
    return [{c: r.get(c) for c in COLUMNS} for r in rows]


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description="fastest cached configurations")
    ap.add_argument("--num-nodes", type=int, required=True)
    ap.add_argument("--gpus-per-node", type=int, required=True)
    ap.add_argument("--gpu-type", required=True, choices=GPUS)
    ap.add_argument("--model", required=True, choices=model_types())
    a = ap.parse_args(argv)
    print_table(optimal_configs(a.num_nodes, a.gpus_per_node, a.gpu_type, a.model), COLUMNS)


if __name__ == "__main__":
    main()
