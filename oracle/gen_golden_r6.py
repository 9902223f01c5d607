"""ORACLE fixture generator, round 6 — run in the build container only (test infrastructure;
nothing here ships or runs on the product path).

Writes tests/golden/fullsize_r6.json (SURVEY.md §8(c)(iii) full-size scalar goldens):

  * `llava-pretrain-train-M<M>` (default M = 32): the reference's own llava-pretrain recipe
    (src/models/llava.py:22-58, 80-124: CLIP-ViT-L/14-336 + Llama-3.2-1B, tower and LLM frozen,
    AdamW lr 1e-3, no clip) on M samples as M / 8 accumulated micro-batches of 8 — projector
    gradient norm, the losses of two AdamW steps and the loss after them, bf16 autocast and
    fp32, and the bf16 rounding noise of every quantity over 12 weight perturbations (VERDICT r05
    #3: the M = 16 record's sigma let its single HF bf16 draw sit 1.1 bars from the HIP value;
    sigma shrinks with M as it did for C2 / C3).

Same machinery as gen_golden_r3.py / r4 / r5 (train_scalars; adam_step_ pinned bitwise to
torch.optim by tests/test_oracle_golden.py; weights oracle.init_params(seed=0), batch
oracle.make_batch(seed=1)).  The oracle restates HF's LlavaForConditionalGeneration(CLIP, Llama)
bit for bit on this model (tests/golden/fullsize_r3.json `oracle_loss_*`).  Resumable: every
finished run is saved.

  * `c5train-M<M>` (GOLDEN_JOB=c5, default M = 8): round 3's C5 training record (M = 2) at
    M samples as M / 2 accumulated micro-batches of 2.

Usage: GOLDEN_THREADS=6 GOLDEN_M=32 python oracle/gen_golden_r6.py
       GOLDEN_JOB=c5 GOLDEN_THREADS=8 GOLDEN_M=8 python oracle/gen_golden_r6.py
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
from oracle.gen_golden_r3 import OUT, _split, c5_cfg, llava_cfg, train_scalars  # noqa: E402
from oracle.gen_golden_r4 import N_SIGMA, _sd_record  # noqa: E402


def c5_train(results: dict, save) -> None:
    """`c5train-M<M>` (default M = 8): BASELINE C5 (CLIP-ViT-L/14-336 +
    Pythia-2.8B @ 576 + 511 tokens) on M samples as M / 2 accumulated micro-batches of 2, AdamW
    lr 1e-4 for two steps, no clip — round 3's `c5train` recipe (gen_golden_r3.py) at 4x the
    samples; Adam moments memory-mapped under $GOLDEN_SCRATCH as there.  GOLDEN_NOISE sets
    the perturbed runs (default 8: 9 samples with the unperturbed run)."""
    M = int(os.environ.get("GOLDEN_M", "8"))
    n_noise = int(os.environ.get("GOLDEN_NOISE", "8"))
    key = f"c5train-M{M}"
    ocfg = c5_cfg()
    batches = _split(O.make_batch(ocfg, M, 511, seed=1), M // 2)
    rec = results.get(key) or {
        "batch": f"oracle.make_batch(seed=1, M={M}, text_len=511) as {M // 2} x 2",
        "weights": "oracle.init_params(seed=0)", "optimizer": "AdamW",
        "betas": [0.9, 0.999], "lrs": [1e-4, 1e-4], "clip": 0.0}
    kw = dict(kind="adamw", lrs=[1e-4, 1e-4], betas=(0.9, 0.999), clip=0.0,
              scratch=os.environ.get("GOLDEN_SCRATCH", "/tmp/mmpt_golden"))
    mk = lambda: O.init_params(ocfg, seed=0)  # noqa: E731
    for prec in ("bf16", "fp32"):
        if prec not in rec:
            t0 = time.time()
            print(f"{key} {prec}", flush=True)
            rec[prec] = train_scalars(mk, ocfg, batches, precision=prec, **kw)
            print(f"  {rec[prec]} ({time.time() - t0:.0f} s)", flush=True)
            results[key] = rec
            save()
    runs = rec.get("noise", {}).get("samples") or [rec["bf16"]]
    while len(runs) < n_noise + 1:
        s = len(runs) - 1
        t0 = time.time()
        runs.append(train_scalars(mk, ocfg, batches, precision="bf16", perturb=s, **kw))
        print(f"  noise run {s}: {runs[-1]} ({time.time() - t0:.0f} s)", flush=True)
        rec["noise"] = _sd_record(runs)
        results[key] = rec
        save()


def main():
    torch.set_num_threads(int(os.environ.get("GOLDEN_THREADS", "6")))
    path = os.path.join(OUT, "fullsize_r6.json")
    try:
        with open(path) as f:
            results = json.load(f)
    except (OSError, ValueError):
        results = {}

    def save():
        import transformers

        results["generator"] = "oracle/gen_golden_r6.py"
        results["transformers"] = transformers.__version__
        with open(path, "w") as f:
            json.dump(results, f, indent=1)

    if os.environ.get("GOLDEN_JOB", "llava") == "c5":
        c5_train(results, save)
        return
    llava_train(results, save)


def llava_train(results: dict, save) -> None:
    M = int(os.environ.get("GOLDEN_M", "32"))
    key = f"llava-pretrain-train-M{M}"
    ocfg = llava_cfg()
    P = O.init_params(ocfg, seed=0)
    batches = _split(O.make_batch(ocfg, M, 511, seed=1), M // 8)
    rec = results.get(key) or {
        "batch": f"oracle.make_batch(seed=1, M={M}, text_len=511) as {M // 8} x 8",
        "weights": "oracle.init_params(seed=0)", "optimizer": "AdamW",
        "betas": [0.9, 0.999], "lrs": [1e-3, 1e-3], "clip": 0.0,
        "trainable": "proj.* (tower and LLM frozen, src/models/llava.py:49-52)"}
    kw = dict(kind="adamw", lrs=[1e-3, 1e-3], betas=(0.9, 0.999), clip=0.0,
              trainable=lambda n: n.startswith("proj."))
    mk = lambda: {k: v.clone() for k, v in P.items()}  # noqa: E731
    for prec in ("bf16", "fp32"):
        if prec not in rec:
            t0 = time.time()
            print(f"{key} {prec}", flush=True)
            rec[prec] = train_scalars(mk, ocfg, batches, precision=prec, **kw)
            print(f"  {rec[prec]} ({time.time() - t0:.0f} s)", flush=True)
            results[key] = rec
            save()
    runs = rec.get("noise", {}).get("samples") or [rec["bf16"]]
    while len(runs) < N_SIGMA + 1:
        s = len(runs) - 1
        t0 = time.time()
        runs.append(train_scalars(mk, ocfg, batches, precision="bf16", perturb=s, **kw))
        print(f"  noise run {s}: {runs[-1]} ({time.time() - t0:.0f} s)", flush=True)
        rec["noise"] = _sd_record(runs)
        results[key] = rec
        save()


if __name__ == "__main__":
    main()
