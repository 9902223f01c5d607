"""Sweeps of the empirical training-time experiment with a local results cache — the
reference's `Sweep` / `TrainingTimeEmpiricalSweep` (experiments/utils/base_classes.py:
141-259, experiments/training_time_empirical_sweep.py:13-38) without ai2-tango, polars,
submitit or torchrunx (none are in this image):

* the cache is one JSON file per experiment under `$MMPT_RESULTS_DIR` (default
  `<repo>/results/`), keyed by a hash of the experiment's fields;
* `run` launches every valid, uncached experiment as ONE `torch.distributed.run` job
  with one process per GPU of this node (`--nproc-per-node gpus_per_node`, rendezvous on
  127.0.0.1); rank 0 writes the result file.  Failed jobs are recorded with
  `training_days = None` (like an OOM in the reference) unless `retry_failed`;
* `count` / `print-incomplete` / `print-results` behave as in the reference.

Child entry point: `python -m multimodal_llm_pretraining_amd.sweep --experiment '<json>'`.
"""

from __future__ import annotations

import argparse
import hashlib
import itertools
import json
import os
import socket
import subprocess
import sys
from dataclasses import dataclass
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent

CONFIG_FIELDS = ("num_nodes", "gpus_per_node", "gpu_type", "model", "free_lunch",
                 "activation_checkpointing", "sharding", "offloading")


def results_dir() -> Path:
    return Path(os.environ.get("MMPT_RESULTS_DIR") or ROOT / "results")


@dataclass
class Experiment:
    """TrainingTimeEmpirical's identity (config + benchmarking_steps + trial) and its
    cache entry; the experiment itself runs in the launched processes."""

    config: dict
    benchmarking_steps: int = 3
    trial: int = 0

    def to_dict(self) -> dict:
        return {**{k: self.config[k] for k in CONFIG_FIELDS},
                "benchmarking_steps": self.benchmarking_steps, "trial": self.trial}

    @property
    def key(self) -> str:
        blob = json.dumps(self.to_dict(), sort_keys=True)
        return hashlib.sha1(blob.encode()).hexdigest()[:16]

    @property
    def path(self) -> Path:
        return results_dir() / "training_time_empirical" / f"{self.key}.json"

    def is_cached(self) -> bool:
        return self.path.exists()

    def results(self) -> dict:
        with open(self.path) as f:
            return json.load(f)["result"]

    def is_valid(self) -> bool:
        from .experiments import TrainingConfig, TrainingTimeEmpirical

        return TrainingTimeEmpirical(TrainingConfig(**self.config), self.benchmarking_steps,
                                     self.trial).is_valid()

    def __str__(self) -> str:
        return "TrainingTimeEmpirical(" + ", ".join(f"{k}={v!r}" for k, v in self.to_dict().items()) + ")"

    # ------------------------------------------------------------ execution
    def command(self, port: int) -> list[str]:
        n = self.config["gpus_per_node"]
        return [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1",
                "--nproc-per-node", str(n), "--master-addr", "127.0.0.1",
                "--master-port", str(port), "-m", "multimodal_llm_pretraining_amd.sweep",
                "--experiment", json.dumps(self.to_dict())]

    def launch(self, timeout: float | None = None) -> bool:
        if self.config["num_nodes"] != 1:
            raise NotImplementedError("multi-node sweeps need a cluster launcher (SLURM is out "
                                      "of scope here); run one node at a time")
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get(
            "HSA_ENABLE_IPC_MODE_LEGACY", "0"))
        env["PYTHONPATH"] = str(ROOT) + os.pathsep + env.get("PYTHONPATH", "")
        rc = subprocess.run(self.command(_free_port()), env=env, cwd=str(ROOT),
                            timeout=timeout).returncode
        if rc != 0 and not self.is_cached():
            self.write({"error": f"exit status {rc}", "training_days": None})
        return rc == 0

    def write(self, result: dict) -> None:
        self.path.parent.mkdir(parents=True, exist_ok=True)
        tmp = self.path.with_suffix(".tmp")
        with open(tmp, "w") as f:
            json.dump({"experiment": self.to_dict(), "result": result}, f, indent=1)
        os.replace(tmp, self.path)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@dataclass
class TrainingTimeEmpiricalSweep:
    search_space: dict
    benchmarking_steps: int = 3
    trial: int = 0

    def __post_init__(self):
        if isinstance(self.search_space, (str, Path)):
            with open(self.search_space) as f:
                self.search_space = json.load(f)

    @property
    def experiments(self) -> list[Experiment]:
        keys = list(self.search_space)
        out = []
        for values in itertools.product(*self.search_space.values()):
            e = Experiment(dict(zip(keys, values)), self.benchmarking_steps, self.trial)
            if e.is_valid():
                out.append(e)
        return out

    @property
    def num_cached(self) -> int:
        return sum(e.is_cached() for e in self.experiments)

    def results(self) -> list[dict]:
        return [{**e.to_dict(), **e.results()} for e in self.experiments if e.is_cached()]

    def print_results(self) -> None:
        print_table(self.results())

    def print_incomplete(self) -> None:
        print("\nThe following experiments are incomplete and are not currently running:\n")
        for e in self.experiments:
            if not e.is_cached():
                print(e)

    def sweep(self, slurm: bool = False, retry_failed: bool = False) -> None:
        if slurm:
            raise NotImplementedError("SLURM submission is out of scope (no cluster here); "
                                      "run the sweep on each node")
        todo = [e for e in self.experiments
                if not e.is_cached() or (retry_failed and e.results().get("error"))]
        for i, e in enumerate(todo):
            print(f"[{i + 1}/{len(todo)}] {e}", flush=True)
            if e.is_cached():
                e.path.unlink()
            e.launch()

    @classmethod
    def run(cls, experiment_sweep: "TrainingTimeEmpiricalSweep", cmd: str = "run",
            slurm: bool = False) -> None:
        if cmd == "run":
            experiment_sweep.sweep(slurm=slurm)
        elif cmd == "count":
            print(f"# cached experiments: {experiment_sweep.num_cached} / "
                  f"{len(experiment_sweep.experiments)}")
        elif cmd == "print-incomplete":
            experiment_sweep.print_incomplete()
        elif cmd == "print-results":
            experiment_sweep.print_results()
        else:
            raise ValueError(f"cmd {cmd!r} not in run/count/print-incomplete/print-results")


def print_table(rows: list[dict], columns: list[str] | None = None) -> None:
    if not rows:
        print("(no results)")
        return
    columns = columns or list(rows[0])
    cells = [[("" if r.get(c) is None else str(r.get(c))) for c in columns] for r in rows]
    width = [max(len(c), *(len(x[i]) for x in cells)) for i, c in enumerate(columns)]
    print("  ".join(c.ljust(w) for c, w in zip(columns, width)))
    print("  ".join("-" * w for w in width))
    for x in cells:
        print("  ".join(v.ljust(w) for v, w in zip(x, width)))


def _child(exp: dict) -> int:
    """One rank of a launched experiment (torch.distributed.run sets RANK/WORLD_SIZE)."""
    import torch
    import torch.distributed as dist

    from .experiments import TrainingConfig, TrainingTimeEmpirical

    local = int(os.environ.get("LOCAL_RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    cfg = {k: exp[k] for k in CONFIG_FIELDS}
    e = Experiment(cfg, exp["benchmarking_steps"], exp["trial"])
    res = TrainingTimeEmpirical(TrainingConfig(**cfg), e.benchmarking_steps, e.trial).run()
    if int(os.environ.get("RANK", "0")) == 0:
        e.write(res)
    if world > 1:
        dist.destroy_process_group()
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--experiment", required=True, help="JSON of Experiment.to_dict()")
    a = ap.parse_args(argv)
    return _child(json.loads(a.experiment))


if __name__ == "__main__":
    sys.exit(main())
