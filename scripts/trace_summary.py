#!/usr/bin/env python
"""Per-(kernel, grid) device time per step from a rocprofv3 kernel_trace CSV.
Usage: python scripts/trace_summary.py <run_kernel_trace.csv> <steps-in-trace> [filter]"""
import collections
import csv
import sys

path, steps = sys.argv[1], float(sys.argv[2])
filt = sys.argv[3] if len(sys.argv) > 3 else ""
agg = collections.defaultdict(lambda: [0, 0.0])
tot = 0.0
for r in csv.DictReader(open(path)):
    n = r["Kernel_Name"].replace("mmpt::(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    if filt and filt not in n:
        continue
    key = (n, r["Grid_Size_X"], r["Grid_Size_Y"])
    agg[key][0] += 1
    agg[key][1] += d
print(f"total device time per step: {tot / steps / 1e3:.1f} ms")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
    print(f"{k[0][:44]:44s} gx={k[1]:>9} gy={k[2]:>4} n={v[0]:5d} avg={v[1] / v[0]:9.1f}us "
          f"per-step={v[1] / steps / 1e3:7.2f}ms")
