#!/usr/bin/env python
"""Fold the parity JSON lines written by the full-size GPU tests (tests/parity_record.py)
into one summary: python scripts/parity_summary.py <jsonl> <out.json>"""

import json
import sys

recs = [json.loads(l) for l in open(sys.argv[1]) if l.strip()]
last = {}
for r in recs:  # the latest record per (test, quantity)
    last[(r["test"], r["quantity"])] = r
rows = sorted(last.values(), key=lambda r: (r["test"], r["quantity"]))
def ratio(r):  # the pass criterion: the nearer of the bf16 and fp32 HF references, over the bar
    d = r["abs_delta"]
    if r.get("abs_delta_fp32") is not None:
        d = min(d, r["abs_delta_fp32"])
    return d / r["tol"]


out = {"source": sys.argv[1], "n": len(rows), "all_pass": all(r["pass"] for r in rows),
       "max_pass_ratio": max(ratio(r) for r in rows) if rows else None,
       "pass_ratio_definition": "min(|HIP - HF bf16|, |HIP - HF fp32|) / bar (the test's "
                                "criterion, tests/parity_record.within)",
       "max_abs_delta_bf16_over_tol": max(r["abs_delta"] / r["tol"] for r in rows) if rows else None,
       "max_abs_z_vs_noise_mean": max((abs(r["hip"] - r["noise_mean"]) / r["sigma"] for r in rows
                                       if r.get("noise_mean") is not None and r.get("sigma")),
                                      default=None),
       "z_definition": "(HIP - mean of the golden's bf16 noise samples) / sigma, where the "
                       "golden keeps its samples",
       "records": rows}
with open(sys.argv[2], "w") as f:
    json.dump(out, f, indent=1)
for r in rows:
    print(f"{r['test']:45s} {r['quantity']:12s} |d| {r['abs_delta']:.2e} tol {r['tol']:.2e} "
          f"ratio {ratio(r):.2f} {'ok' if r['pass'] else 'FAIL'}")
