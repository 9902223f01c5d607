"""Check that a committed rocprofv3 kernel-trace summary reproduces the bench line it was
taken with: for every GEMM shape of the line's `roofline.gemm_shapes`
table, the rocprof average duration of that kernel name over the launches of the timed
region vs the line's HIP-event average.

rocprof aggregates by kernel NAME, the line by (name, M, N, K, epilogue): names shared by
several shapes are compared as a launch-weighted mean of the line's shapes.  The traced
command runs warm-up + timed steps; the line's table covers only the timed steps, so the
rocprof average includes the warm-up launches of the same shapes (same work per launch).

Usage: python scripts/diag/prof_vs_line.py <trace_bench.json> <run_kernel_stats.csv> [out.json]
"""

from __future__ import annotations

import csv
import json
import sys


def main():
    line = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    stats = {r["Name"]: r for r in csv.DictReader(open(sys.argv[2]))}
    shapes = line["roofline"]["gemm_shapes"]
    steps = line["steps"]
    by_name: dict[str, list] = {}
    for s in shapes:
        a = by_name.setdefault(s["kernel"], [0.0, 0.0])
        n = s["launches_per_step"] * steps
        a[0] += n * s["avg_us"]
        a[1] += n
    rows = []
    for name, (us_n, n) in sorted(by_name.items(), key=lambda kv: -kv[1][0]):
        hits = [r for k, r in stats.items() if name in k.replace("mmpt::(anonymous namespace)::", "")]
        if not hits:
            rows.append({"kernel": name, "line_avg_us": round(us_n / n, 1), "rocprof_avg_us": None})
            continue
        tot = sum(float(r["TotalDurationNs"]) for r in hits)
        calls = sum(int(r["Calls"]) for r in hits)
        prof = tot / calls / 1e3
        line_us = us_n / n
        rows.append({"kernel": name, "line_launches": int(n), "line_avg_us": round(line_us, 1),
                     "rocprof_calls": calls, "rocprof_avg_us": round(prof, 1),
                     "rel_diff": round(prof / line_us - 1, 4)})
    dom = line["roofline"]["kernel"]
    out = {"line": sys.argv[1], "stats": sys.argv[2], "dominant": dom,
           "dominant_rel_diff": next((r.get("rel_diff") for r in rows if r["kernel"] == dom), None),
           "note": "rocprof averages include the warm-up steps' launches; the line's only the "
                   "timed steps' (same shapes, same work per launch)",
           "kernels": rows}
    s = json.dumps(out, indent=1)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
