"""The drop-in scripts on the GPU: scripts/training.py driven by a TrainingArguments JSON
(plain DDP-style and the ZeRO-3 + gradient-checkpointing DeepSpeed block), and one
experiment of the scripts/benchmark.py sweep through its torch.distributed.run launch
(results cache + scripts/print_optimal_config.py)."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

pytestmark = pytest.mark.gpu

BASE = {"max_steps": 1430, "per_device_train_batch_size": 2, "gradient_accumulation_steps": 2,
        "lr_scheduler_type": "cosine_with_min_lr", "lr_scheduler_kwargs": {"min_lr_rate": 0.1},
        "warmup_steps": 1, "gradient_checkpointing": False, "bf16": True, "fp16": False,
        "tf32": False, "fsdp": "", "fsdp_config": None, "deepspeed": None,
        "ddp_find_unused_parameters": False, "torch_compile": True, "max_grad_norm": 1.0}


@pytest.mark.parametrize("extra", [{}, {"gradient_checkpointing": True,
                                        "deepspeed": {"zero_optimization": {"stage": 3}}}])
def test_training_script_steps(tmp_path, extra):
    from training import train

    log = train(str(tmp_path), "pythia-160m", {**BASE, **extra}, max_steps=4)
    assert [r["step"] for r in log] == [1, 2, 3, 4]
    assert log[0]["learning_rate"] == 0.0  # warmup step 0
    assert log[-1]["loss"] < log[1]["loss"]
    lines = open(tmp_path / "trainer_log.jsonl").read().splitlines()
    assert len(lines) == 4 and json.loads(lines[-1])["step"] == 4


def test_sweep_runs_one_experiment(tmp_path):
    env = dict(os.environ, MMPT_RESULTS_DIR=str(tmp_path))
    cmd = [sys.executable, "scripts/benchmark.py", "--num-nodes", "1", "--gpus-per-node", "1",
           "--gpu-type", "mi355x", "--model", "vit-b16-pythia-1b", "--methods", "naive"]
    out = subprocess.run(cmd + ["--cmd", "run"], cwd=ROOT, env=env, capture_output=True, text=True,
                         timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    files = list((tmp_path / "training_time_empirical").glob("*.json"))
    assert len(files) == 1
    res = json.load(open(files[0]))["result"]
    assert res.get("training_days") is not None, res
    assert res["micro_batch_size"] >= 1 and res["step_time"] > 0
    out = subprocess.run([sys.executable, "scripts/print_optimal_config.py", "--num-nodes", "1",
                          "--gpus-per-node", "1", "--gpu-type", "mi355x", "--model", "vit-b16-pythia-1b"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and "vit-b16-pythia-1b" in out.stdout
