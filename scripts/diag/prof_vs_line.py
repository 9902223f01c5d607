"""Check that a committed rocprofv3 kernel-trace summary reproduces the bench line it was
taken with: for every GEMM shape of the line's `roofline.gemm_shapes`
table, the rocprof average duration of that kernel name over the launches of the timed
region vs the line's HIP-event average.

rocprof aggregates by kernel NAME, the line by (name, M, N, K, epilogue): names shared by
several shapes are compared as a launch-weighted mean of the line's shapes.  The traced
command runs warm-up + timed steps and the line's table covers only the timed steps: with the
per-dispatch trace (run_kernel_trace.csv) the last n dispatches of each kernel are compared
(the warm-up steps run at a lower clock), else the summary's all-dispatch average.

Usage: python scripts/diag/prof_vs_line.py <trace_bench.json> <run_kernel_stats.csv> [out.json]
"""

from __future__ import annotations

import csv
import json
import os
import sys


def main():
    line = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    stats = {r["Name"]: r for r in csv.DictReader(open(sys.argv[2]))}
    shapes = line["roofline"]["gemm_shapes"]
    steps = line["steps"]
    by_name: dict[str, list] = {}
    for s in shapes:
        if s.get("overlapped"):  # weight-gradient stream launches carry no rate (round 6)
            continue
        a = by_name.setdefault(s["kernel"], [0.0, 0.0])
        n = s["launches_per_step"] * steps
        a[0] += n * s["avg_us"]
        a[1] += n
    # the per-dispatch trace beside the summary, when present: the LAST n dispatches of each
    # kernel are the timed region's (the warm-up steps come first; traced runs have no
    # yardstick), so the comparison covers exactly the launches the line averaged
    trace = os.path.join(os.path.dirname(sys.argv[2]), "run_kernel_trace.csv")
    disp: dict[str, list] = {}
    opener = open
    if not os.path.exists(trace) and os.path.exists(trace + ".gz"):  # (committed copies)
        import gzip

        trace, opener = trace + ".gz", lambda f: gzip.open(f, "rt")
    if os.path.exists(trace):
        for r in csv.DictReader(opener(trace)):
            nm = r["Kernel_Name"].replace("mmpt::(anonymous namespace)::", "")
            disp.setdefault(nm, []).append((int(r["Start_Timestamp"]),
                                            int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows = []
    for name, (us_n, n) in sorted(by_name.items(), key=lambda kv: -kv[1][0]):
        line_us = us_n / n
        d = sorted(x for k, v in disp.items() if name in k for x in v)
        if d:
            last = d[-int(round(n)):]
            prof = sum(x[1] for x in last) / len(last) / 1e3
            rows.append({"kernel": name, "line_launches": int(n), "line_avg_us": round(line_us, 1),
                         "rocprof_dispatches": len(last), "rocprof_avg_us": round(prof, 1),
                         "rocprof_all_dispatches_avg_us": round(sum(x[1] for x in d) / len(d) / 1e3, 1),
                         "rel_diff": round(prof / line_us - 1, 4), "basis": "last n dispatches (timed steps)"})
            continue
        hits = [r for k, r in stats.items() if name in k.replace("mmpt::(anonymous namespace)::", "")]
        if not hits:
            rows.append({"kernel": name, "line_avg_us": round(line_us, 1), "rocprof_avg_us": None})
            continue
        tot = sum(float(r["TotalDurationNs"]) for r in hits)
        calls = sum(int(r["Calls"]) for r in hits)
        prof = tot / calls / 1e3
        rows.append({"kernel": name, "line_launches": int(n), "line_avg_us": round(line_us, 1),
                     "rocprof_calls": calls, "rocprof_avg_us": round(prof, 1),
                     "rel_diff": round(prof / line_us - 1, 4), "basis": "summary (all dispatches)"})
    dom = line["roofline"]["kernel"]
    out = {"line": sys.argv[1], "stats": sys.argv[2], "dominant": dom,
           "dominant_rel_diff": next((r.get("rel_diff") for r in rows if r["kernel"] == dom), None),
           "note": "with run_kernel_trace.csv beside the summary: the last n dispatches of each "
                   "kernel (the timed steps'); else the summary's average over every dispatch "
                   "(warm-up included)",
           "kernels": rows}
    s = json.dumps(out, indent=1)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
