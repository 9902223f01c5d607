#!/usr/bin/env python
"""Summarise rocprofv3 PMC passes into HBM bytes per launch, per kernel.

Inputs: the FETCH_SIZE and WRITE_SIZE counter_collection CSVs of two separate
`rocprofv3 --pmc` passes over the same bench command (scripts/diag/gpu_profile.sh; the two
counters cannot share a pass on gfx950).  Corrections per MI355X_MICROARCH.md
§HBM: FETCH_SIZE (KiB) reports half the bytes of wide coalesced reads on gfx950 ->
doubled; WRITE_SIZE (KiB) is exact for 16-B-per-lane stores.

Usage: python scripts/pmc_traffic.py <fetch.csv> <write.csv> <tag> --workload MODEL|mbsM|SHARDING
       [-o profiles/pmc_traffic.json]   (merged into the file under that workload key: the
       bench line only quotes traffic measured on its own workload)
"""

from __future__ import annotations

import argparse
import csv
import json
import re
from collections import defaultdict

NAME = re.compile(r"(\w+_kernel<[^>]*>|\w+_kernel\b|\w+(?=\())")


def short(name: str) -> str:
    name = name.replace("mmpt::(anonymous namespace)::", "")
    m = NAME.search(name.replace("void ", "", 1))
    return m.group(1) if m else name


def per_kernel(path: str, counter: str) -> dict[str, list[float]]:
    out: dict[str, list[float]] = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter:
                out[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("tag")
    ap.add_argument("--workload", required=True, help="bench workload key, e.g. vit-b16-pythia-1b|mbs256|ddp")
    ap.add_argument("-o", default="profiles/pmc_traffic.json")
    args = ap.parse_args()
    fetch = per_kernel(args.fetch, "FETCH_SIZE")
    write = per_kernel(args.write, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) & set(write)):
        f = sum(fetch[k]) / len(fetch[k]) * 1024 * 2  # KiB -> B, gfx950 x2 correction
        w = sum(write[k]) / len(write[k]) * 1024
        kernels[k] = {"launches": len(fetch[k]), "fetch_bytes_per_launch": round(f),
                      "write_bytes_per_launch": round(w), "hbm_bytes_per_launch": round(f + w),
                      "source": f"{args.tag}: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes"}
    try:
        with open(args.o) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        rec = {"note": "HBM bytes per launch from rocprofv3 PMC (FETCH_SIZE x2 gfx950 correction, "
                       "MI355X_MICROARCH.md §HBM); one pass per counter over the same bench "
                       "command; keyed by workload (model|micro-batch|sharding), then kernel",
               "workloads": {}}
    rec.setdefault("workloads", {})[args.workload] = {"tag": args.tag, "kernels": kernels}
    with open(args.o, "w") as f:
        json.dump(rec, f, indent=1)
    for k, v in kernels.items():
        print(f"{k:40s} {v['launches']:5d} fetch {v['fetch_bytes_per_launch']/1e6:9.1f} MB "
              f"write {v['write_bytes_per_launch']/1e6:9.1f} MB")


if __name__ == "__main__":
    main()
