"""ORACLE fixture generator, round 5 — run in the build container only (test infrastructure;
nothing here ships or runs on the product path).

Writes tests/golden/fullsize_r5.json (SURVEY.md §8(c)(iii) full-size scalar goldens):

  * `c2train-M16`: BASELINE C2 (Pythia-1B @ 2049 tokens, Adam betas (0.9, 0.95), clip 1.0,
    src/models/pythia.py:44-78) at M = 16 — run as 8 accumulated micro-batches of 2, the loss
    normaliser the label count of the whole step (HF num_items_in_batch): step-1 gradient L2
    norm, the losses of two Adam steps (lr 1e-4) and the loss after them, bf16 autocast and
    fp32, and the bf16 rounding noise σ of every quantity over 12 weight perturbations
    (VERDICT r04 "next" #6: the M = 1 C2 record's σ, 6.3e-4 on the loss after two steps, let a
    1e-3 optimizer-path regression pass; σ shrinks with M as it did for C3).

Same machinery as gen_golden_r3.py / r4 (train_scalars; adam_step_ pinned bitwise to
torch.optim by tests/test_oracle_golden.py; weights oracle.init_params(seed=0), batch
oracle.make_batch(seed=1)).  Resumable: every finished run is saved.

Usage: GOLDEN_THREADS=6 python oracle/gen_golden_r5.py
"""

from __future__ import annotations

import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

from oracle import model as O  # noqa: E402
from oracle.gen_golden_r3 import OUT, _split, c2_cfg, train_scalars  # noqa: E402
from oracle.gen_golden_r4 import N_SIGMA, _sd_record  # noqa: E402


def main():
    torch.set_num_threads(int(os.environ.get("GOLDEN_THREADS", "6")))
    path = os.path.join(OUT, "fullsize_r5.json")
    try:
        with open(path) as f:
            results = json.load(f)
    except (OSError, ValueError):
        results = {}

    def save():
        import transformers

        results["generator"] = "oracle/gen_golden_r5.py"
        results["transformers"] = transformers.__version__
        with open(path, "w") as f:
            json.dump(results, f, indent=1)

    ocfg = c2_cfg()
    batches = _split(O.make_batch(ocfg, 16, 2049, seed=1), 8)
    rec = results.get("c2train-M16") or {
        "batch": "oracle.make_batch(seed=1, M=16, text_len=2049) as 8 x 2",
        "weights": "oracle.init_params(seed=0)", "optimizer": "Adam",
        "betas": [0.9, 0.95], "lrs": [1e-4, 1e-4], "clip": 1.0}
    kw = dict(kind="adam", lrs=[1e-4, 1e-4], betas=(0.9, 0.95), clip=1.0)
    mk = lambda: O.init_params(ocfg, seed=0)  # noqa: E731
    for prec in ("bf16", "fp32"):
        if prec not in rec:
            t0 = time.time()
            print(f"c2train-M16 {prec}", flush=True)
            rec[prec] = train_scalars(mk, ocfg, batches, precision=prec, **kw)
            print(f"  {rec[prec]} ({time.time() - t0:.0f} s)", flush=True)
            results["c2train-M16"] = rec
            save()
    runs = rec.get("noise", {}).get("samples") or [rec["bf16"]]
    while len(runs) < N_SIGMA + 1:
        s = len(runs) - 1
        t0 = time.time()
        runs.append(train_scalars(mk, ocfg, batches, precision="bf16", perturb=s, **kw))
        print(f"  noise run {s}: {runs[-1]} ({time.time() - t0:.0f} s)", flush=True)
        rec["noise"] = _sd_record(runs)
        results["c2train-M16"] = rec
        save()


if __name__ == "__main__":
    main()
