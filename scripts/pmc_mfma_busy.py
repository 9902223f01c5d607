#!/usr/bin/env python
"""MFMA-busy fraction per launch from scripts/diag/gemm_pmc.sh / attn_pmc.sh output: joins the
`sq` pass (SQ_VALU_MFMA_BUSY_CYCLES, summed over the chip's SIMDs) with the `tcc` pass
(GRBM_GUI_ACTIVE, summed over the 8 XCDs) by dispatch order, and reports
busy / (SIMDs × GRBM/8) and the effective clock GRBM/8 / duration per kernel launch.

python scripts/pmc_mfma_busy.py <pmc dir> [--simds 1024] [--labels a,b,c --per-label 6]"""

import argparse
import collections
import csv
import os


def load(path):
    out = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        key = (int(r["Dispatch_Id"]), r["Kernel_Name"])
        d = out.setdefault(key, {"dur_us": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return list(out.items())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--simds", type=int, default=1024)
    ap.add_argument("--labels", default="")
    ap.add_argument("--per-label", type=int, default=6)
    a = ap.parse_args()
    sq = load(os.path.join(a.dir, "sq", "run_counter_collection.csv"))
    tcc = load(os.path.join(a.dir, "tcc", "run_counter_collection.csv"))
    labels = a.labels.split(",") if a.labels else []
    n = min(len(sq), len(tcc))
    print(f"{'#':>3s} {'label':16s} {'kernel':44s} {'us':>9s} {'clock GHz':>9s} {'MFMA busy':>9s}")
    for i in range(n):
        (_, name), s = sq[i]
        (_, name2), t = tcc[i]
        if name != name2:
            continue
        k = name.replace("mmpt::(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        cyc = t.get("GRBM_GUI_ACTIVE", 0.0) / 8
        busy = s.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (a.simds * cyc) if cyc else 0.0
        clk = cyc / (t["dur_us"] * 1e3) if t["dur_us"] else 0.0
        lab = labels[i // a.per_label] if i // a.per_label < len(labels) else ""
        print(f"{i:3d} {lab:16s} {k[:44]:44s} {t['dur_us']:9.1f} {clk:9.2f} {busy:9.3f}")


if __name__ == "__main__":
    main()
