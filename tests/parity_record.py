"""Achieved parity deltas of the full-size GPU tests, appended as JSON lines so a run leaves a
record of how close the HIP step is (the deltas were only printed).  The file is
$MMPT_PARITY_OUT, default gpurun_out/parity/parity_deltas.jsonl under the repo root (gpurun
copies gpurun_out/ back); scripts/parity_summary.py folds it into
profiles/<round>/parity_deltas.json."""

import json
import os
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def bar(sigma: float, k: float = 2.0) -> float:
    """The full-size bar: the north-star 1e-4 absolute plus k times the quantity's measured
    bf16 rounding-noise sigma (tests/golden/fullsize_*.json)."""
    return 1e-4 + k * sigma


def record(test: str, quantity: str, got: float, ref: float, tol: float, **extra) -> None:
    path = os.environ.get("MMPT_PARITY_OUT") or os.path.join(ROOT, "gpurun_out", "parity",
                                                             "parity_deltas.jsonl")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    rec = {"test": test, "quantity": quantity, "hip": got, "ref_bf16": ref, "delta": got - ref,
           "abs_delta": abs(got - ref), "tol": tol, "pass": abs(got - ref) < tol,
           "time": time.strftime("%Y-%m-%dT%H:%M:%S"), **extra}
    with open(path, "a") as f:
        f.write(json.dumps(rec) + "\n")
    print(f"  {test} {quantity}: HIP {got:.7f} HF bf16 {ref:.7f} |d| {abs(got - ref):.2e} "
          f"tol {tol:.2e}", flush=True)
