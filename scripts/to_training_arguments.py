#!/usr/bin/env python
"""scripts/to_training_arguments.py of the reference (argparse instead of tyro):
write the HF TrainingArguments dict of a TrainingConfig + micro-batch/GA to JSON.

python scripts/to_training_arguments.py --output args.json --num-nodes 1 --gpus-per-node 8 \
    --gpu-type mi355x --model vit-b16-pythia-1b --micro-batch-size 32 --gradient-accumulation-steps 1
"""

from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from multimodal_llm_pretraining_amd.experiments import SHARDINGS, TrainingConfig  # noqa: E402
from multimodal_llm_pretraining_amd.gpus import GPUS  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--output", type=Path, required=True)
    ap.add_argument("--micro-batch-size", type=int, required=True)
    ap.add_argument("--gradient-accumulation-steps", type=int, required=True)
    ap.add_argument("--num-nodes", type=int, required=True)
    ap.add_argument("--gpus-per-node", type=int, required=True)
    ap.add_argument("--gpu-type", choices=GPUS, required=True)
    ap.add_argument("--model", required=True)
    ap.add_argument("--free-lunch", action="store_true")
    ap.add_argument("--activation-checkpointing", action="store_true")
    ap.add_argument("--sharding", choices=SHARDINGS, default="")
    ap.add_argument("--offloading", action="store_true")
    a = ap.parse_args(argv)
    cfg = TrainingConfig(a.num_nodes, a.gpus_per_node, a.gpu_type, a.model, a.free_lunch,
                         a.activation_checkpointing, a.sharding, a.offloading)
    tc = cfg.training_class(micro_batch_size=a.micro_batch_size,
                            gradient_accumulation_steps=a.gradient_accumulation_steps)
    a.output.parent.mkdir(parents=True, exist_ok=True)
    with open(a.output, "w") as f:
        json.dump(tc._to_huggingface_args_dict(), f)


if __name__ == "__main__":
    main()
