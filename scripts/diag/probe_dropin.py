"""Probe: torch.optim.AdamW over MMPTForPretraining parameter views vs fused Adam."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_dropin_gpu import _tiny  # noqa: E402

from oracle import model as O  # noqa: E402
from multimodal_llm_pretraining_amd.optim import AdamConfig, FusedAdam  # noqa: E402

m, ocfg, P = _tiny()
bd = {k: v.cuda() for k, v in O.make_batch(ocfg, 2, 40, seed=3).items()}
with torch.no_grad():
    l0 = m(**bd).loss.item()
m(**bd).loss.backward()
grads = m.store.grad.clone()
v0 = m.store.master._version
opt = torch.optim.AdamW(m.parameters(), lr=1e-3, weight_decay=0.0, foreach=True)
opt.step()
print("version", v0, "->", m.store.master._version, "recorded", m._shadow_version)
with torch.no_grad():
    l1 = m(**bd).loss.item()
sh_auto = m.store.shadow.clone()
m.store.refresh_shadow()
print("shadow changed by forced refresh:", (m.store.shadow.float() - sh_auto.float()).abs().max().item())
with torch.no_grad():
    l1f = m(**bd).loss.item()
m2, _, _ = _tiny()
m2.store.grad.copy_(grads)
fa = FusedAdam(m2.store.master, m2.store.grad, m2.store.shadow, AdamConfig(lr=1e-3))
fa.step(1e-3)
m2.store.refresh_transposed()
print("master diff", (m2.store.master - m.store.master).abs().max().item(),
      "shadow diff", (m2.store.shadow.float() - m.store.shadow.float()).abs().max().item(),
      "n shadow diff", int((m2.store.shadow != m.store.shadow).sum()))
with torch.no_grad():
    l2 = m2(**bd).loss.item()
print(f"loss before {l0:.6f} torch-auto {l1:.6f} torch-forced {l1f:.6f} fused {l2:.6f}")
d = (m2.store.master - m.store.master).abs()
i = int(d.argmax())
for n, o in m.store.offsets.items():
    if o <= i < o + m.store.p(n).numel():
        print("worst master diff in", n, "value", m.store.master[i].item(), m2.store.master[i].item(),
              "grad", grads[i].item())
