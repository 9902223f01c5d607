"""Effective clock per kernel from a rocprofv3 --pmc GRBM_GUI_ACTIVE pass
(MI355X_MICROARCH.md 'DVFS give-back': GRBM_GUI_ACTIVE is summed over the 8 XCDs, so the
clock is GRBM / 8 / the dispatch's wall time; reads high below ~0.3 ms dispatches).

usage: python scripts/diag/eff_clock.py <run_counter_collection.csv> [--match gemm]"""
import csv
import json
import statistics
import sys


def main():
    path = sys.argv[1]
    match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else ""
    per = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
            continue
        name = r["Kernel_Name"].replace("void ", "").replace("mmpt::(anonymous namespace)::", "")
        name = name.split("(")[0]
        if match and match not in name:
            continue
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        if dur < 3e-4:
            continue
        per.setdefault(name, []).append((float(r["Counter_Value"]) / 8 / dur / 1e6, dur * 1e6))
    out = {n: {"launches": len(v), "eff_clock_mhz_median": round(statistics.median(c for c, _ in v), 1),
               "avg_us": round(sum(d for _, d in v) / len(v), 1)} for n, v in sorted(per.items())}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
