"""Per-tensor gradient comparison at full size (C2: Pythia-1B @ 2049, M = 1): the HIP step vs
the oracle's CPU bf16-autocast and fp32 gradients — which tensors move the global grad norm.
python scripts/diag/diag_gradnorm.py [model] [M] [text_len]"""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

from oracle import model as O  # noqa: E402
from test_parity_gpu import oracle_cfg  # noqa: E402

from multimodal_llm_pretraining_amd import config as C  # noqa: E402
from multimodal_llm_pretraining_amd.engine import Batch, Engine  # noqa: E402
from multimodal_llm_pretraining_amd.params import ParamStore  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "pythia-1b"
M = int(sys.argv[2]) if len(sys.argv) > 2 else 1
L = int(sys.argv[3]) if len(sys.argv) > 3 else 2049
torch.set_num_threads(min(16, os.cpu_count() or 8))
cfg = C.get_config(name)
ocfg = oracle_cfg(cfg)
P = O.init_params(ocfg, seed=0)
batch = O.make_batch(ocfg, M, L, seed=1)
store = ParamStore(C.param_shapes(cfg), "cuda")
store.load(P)
store.refresh_shadow()
eng = Engine(cfg, store)
b = Batch(cfg, batch["input_ids"], batch["labels"], batch.get("pixel_values"), store.device)
eng.forward(b, 1.0 / b.num_items)
eng.backward(b)
torch.cuda.synchronize()
G = {k: store.g(k).cpu() for k in P}
ref = {}
for prec in ("bf16", "fp32"):
    Pr = {k: v.clone().requires_grad_() for k, v in P.items()}
    loss = O.forward_loss(Pr, ocfg, batch, prec)
    loss.backward()
    ref[prec] = {k: v.grad for k, v in Pr.items()}
    print(prec, "loss", loss.item(), flush=True)
    del Pr
tot = {k: sum(float(g.double().pow(2).sum()) for g in d.values()) ** 0.5 for k, d in
       (("hip", G), ("bf16", ref["bf16"]), ("fp32", ref["fp32"]))}
print("global norms", tot)
rows = []
for k in P:
    g, r16, r32 = G[k].double(), ref["bf16"][k].double(), ref["fp32"][k].double()
    rows.append((float(g.pow(2).sum() - r16.pow(2).sum()), k, float(g.norm()), float(r16.norm()),
                 float(r32.norm()), float((g - r16).norm() / (r16.norm() + 1e-30)),
                 float((r16 - r32).norm() / (r32.norm() + 1e-30))))
rows.sort(key=lambda r: -abs(r[0]))
print(f"{'tensor':40s} {'d(sumsq)':>10s} {'|hip|':>10s} {'|bf16|':>10s} {'|fp32|':>10s} "
      f"{'rel(hip,bf16)':>13s} {'rel(bf16,fp32)':>14s}")
for d, k, a, bb, c, e1, e2 in rows[:25]:
    print(f"{k:40s} {d:10.3e} {a:10.5f} {bb:10.5f} {c:10.5f} {e1:13.3e} {e2:14.3e}")
