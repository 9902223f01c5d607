"""ORACLE fixture generator, round 4 — run in the build container only (test infrastructure;
nothing here ships or runs on the product path).

Writes tests/golden/fullsize_r4.json (SURVEY.md §8(c)(iii) full-size scalar goldens):

  * `c3train-M64`: BASELINE C3 (ViT-B/16 + Pythia-1B @ 196 + 511 tokens) at the bench's own
    micro-batch, M = 64, run as 8 accumulated micro-batches of 8 (the loss normaliser is the
    label count of the whole step, HF num_items_in_batch): step-1 gradient L2 norm, the losses
    of two AdamW steps (lr 1e-4) and the loss after them, bf16 autocast and fp32, and the bf16
    rounding noise σ of every quantity over 12 weight perturbations (the M = 16
    training records' σ is 3-4x larger than the bare 1e-4 bar; at M = 64 it should not be).
  * `sigma12`: σ of the round-3 records that sat closest to their bar (llava-pretrain M = 2
    forward loss, llava-pretrain projector training, C5 ZeRO-3 + offload training) re-measured
    with >= 12 perturbations — the round-3 samples are kept and new ones appended
    (perturbation seeds continue where round 3 stopped).

Same machinery as gen_golden_r3.py (train_scalars, adam_step_ pinned bitwise to torch.optim by
tests/test_oracle_golden.py; weights oracle.init_params(seed=0), batches
oracle.make_batch(seed=1)).

Usage: GOLDEN_ONLY=c3m64|sigma12 GOLDEN_THREADS=6 python oracle/gen_golden_r4.py
"""

from __future__ import annotations

import json
import os
import statistics
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

from oracle import model as O  # noqa: E402
from oracle.gen_golden_r3 import (OUT, REL, _perturb_, _split, c3_cfg, c5_cfg,  # noqa: E402
                                  llava_cfg, train_scalars)

N_SIGMA = 12


def _sd_record(runs: list[dict]) -> dict:
    sd = statistics.stdev
    return {"grad_norm": sd([r["grad_norm"] for r in runs]),
            "losses": [sd([r["losses"][i] for r in runs]) for i in range(len(runs[0]["losses"]))],
            "loss_after": sd([r["loss_after"] for r in runs]), "n": len(runs), "rel": REL,
            "definition": "sample std over the unperturbed bf16 run and the weight "
                          "perturbations w*(1 + rel*N(0,1))",
            "samples": runs}


def main():
    torch.set_num_threads(int(os.environ.get("GOLDEN_THREADS", "6")))
    path = os.path.join(OUT, "fullsize_r4.json")
    try:
        with open(path) as f:
            results = json.load(f)
    except (OSError, ValueError):
        results = {}

    def save():
        import transformers

        results["generator"] = "oracle/gen_golden_r4.py"
        results["transformers"] = transformers.__version__
        with open(path, "w") as f:
            json.dump(results, f, indent=1)

    only = os.environ.get("GOLDEN_ONLY", "")
    scratch = os.environ.get("GOLDEN_SCRATCH", "/tmp/mmpt_golden")
    if only in ("", "c3m64"):
        ocfg = c3_cfg()
        batches = _split(O.make_batch(ocfg, 64, 511, seed=1), 8)
        rec = results.get("c3train-M64") or {
            "batch": "oracle.make_batch(seed=1, M=64, text_len=511) as 8 x 8",
            "weights": "oracle.init_params(seed=0)", "optimizer": "AdamW",
            "betas": [0.9, 0.999], "lrs": [1e-4, 1e-4], "clip": 0.0}
        kw = dict(kind="adamw", lrs=[1e-4, 1e-4], betas=(0.9, 0.999), clip=0.0)
        mk = lambda: O.init_params(ocfg, seed=0)  # noqa: E731
        for prec in ("bf16", "fp32"):
            if prec not in rec:
                t0 = time.time()
                print(f"c3train-M64 {prec}", flush=True)
                rec[prec] = train_scalars(mk, ocfg, batches, precision=prec, **kw)
                print(f"  {rec[prec]} ({time.time() - t0:.0f} s)", flush=True)
                results["c3train-M64"] = rec
                save()
        runs = rec.get("noise", {}).get("samples") or [rec["bf16"]]
        while len(runs) < N_SIGMA + 1:
            s = len(runs) - 1
            t0 = time.time()
            runs.append(train_scalars(mk, ocfg, batches, precision="bf16", perturb=s, **kw))
            print(f"  noise run {s}: {runs[-1]} ({time.time() - t0:.0f} s)", flush=True)
            rec["noise"] = _sd_record(runs)
            results["c3train-M64"] = rec
            save()
    if only in ("", "sigma12"):
        with open(os.path.join(OUT, "fullsize_r3.json")) as f:
            r3 = json.load(f)
        sig = results.setdefault("sigma12", {})
        # llava-pretrain M = 2 forward loss: population std over the perturbations, as r3
        if "llava-pretrain" not in sig:
            ocfg = llava_cfg()
            P = O.init_params(ocfg, seed=0)
            batch = O.make_batch(ocfg, 2, 511, seed=1)
            out = []
            with torch.no_grad():
                for s in range(16):
                    P2 = {k: v.clone() for k, v in P.items()}
                    _perturb_(P2, s)
                    out.append(O.forward_loss(P2, ocfg, batch, "bf16").item())
                    del P2
                    print(f"  llava fwd noise {s}: {out[-1]}", flush=True)
            sig["llava-pretrain"] = {"bf16_noise_std": statistics.pstdev(out), "n": len(out),
                                     "samples": out, "rel": REL}
            save()
        jobs = {
            "llava-pretrain-train": (llava_cfg, lambda o: _split(O.make_batch(o, 16, 511, seed=1), 2),
                                     dict(kind="adamw", lrs=[1e-3, 1e-3], betas=(0.9, 0.999),
                                          clip=0.0, trainable=lambda n: n.startswith("proj."))),
            "c5train": (c5_cfg, lambda o: [O.make_batch(o, 2, 511, seed=1)],
                        dict(kind="adamw", lrs=[1e-4, 1e-4], betas=(0.9, 0.999), clip=0.0,
                             scratch=scratch)),
        }
        for key, (mkcfg, mkb, kw) in jobs.items():
            # round 3 kept the samples of c5train, not of llava-pretrain-train (n = 4, seeds
            # 0-2): that one restarts from the unperturbed bf16 run (same seeds, same values)
            old = r3[key]["noise"].get("samples") or [r3[key]["bf16"]]
            runs = sig.get(key, {}).get("samples") or list(old)
            ocfg = mkcfg()
            batches = mkb(ocfg)
            while len(runs) < N_SIGMA + 1:
                s = len(runs) - 1  # r3 drew seeds 0 .. len(old) - 2
                t0 = time.time()
                runs.append(train_scalars(lambda: O.init_params(ocfg, seed=0), ocfg, batches,
                                          precision="bf16", perturb=s, **kw))
                print(f"  {key} noise run {s}: {runs[-1]} ({time.time() - t0:.0f} s)", flush=True)
                sig[key] = _sd_record(runs)
                save()


if __name__ == "__main__":
    main()
