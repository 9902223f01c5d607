#!/usr/bin/env python
"""Print per-kernel averages of every counter in rocprofv3 counter_collection CSVs.

Usage: python scripts/pmc_summary.py <counter_collection.csv> [...]
"""

from __future__ import annotations

import csv
import sys
from collections import defaultdict


def main():
    vals: dict = defaultdict(lambda: defaultdict(list))
    dur: dict = defaultdict(list)
    for path in sys.argv[1:]:
        with open(path) as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"].replace("mmpt::(anonymous namespace)::", "").split("(")[0]
                k = k.replace("void ", "") + f" grid={r['Grid_Size']}"
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                if r["Counter_Name"] == next(iter(vals[k])):
                    dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, cs in vals.items():
        d = dur[k]
        print(f"== {k}  launches={len(d)}  avg_us={sum(d) / max(1, len(d)):.1f}")
        for c, v in sorted(cs.items()):
            print(f"   {c:28s} {sum(v) / len(v):16.1f}")


if __name__ == "__main__":
    main()
