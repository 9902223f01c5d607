"""Diagnostic: GPU vs CPU-oracle loss for head_dim 80 (padded D=128 attention) at growing
batch sizes — a bias would persist while the bf16 rounding noise shrinks."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_parity_gpu import gpu_setup, oracle_cfg  # noqa: E402

from multimodal_llm_pretraining_amd import config as C  # noqa: E402
from multimodal_llm_pretraining_amd.engine import Batch  # noqa: E402
from oracle import model as O  # noqa: E402

import sys as _s
NAMES = _s.argv[1:] or ["tiny-lm", "tiny-lm-d80"]
for name in NAMES:
    ocfg = oracle_cfg(C.get_config(name))
    P = O.init_params(ocfg, seed=0)
    cfg, store, eng = gpu_setup(name, P)
    for M in (2, 8, 32):
        batch = O.make_batch(ocfg, M, 258 if ocfg.vision is None else 47, seed=1)
        with torch.no_grad():
            f32 = O.forward_loss(P, ocfg, batch, "fp32").item()
            b16 = O.forward_loss(P, ocfg, batch, "bf16").item()
        b = Batch(cfg, batch["input_ids"], batch["labels"], batch.get("pixel_values"), store.device)
        g = eng.forward(b, 1.0 / b.num_items, need_grad=False).item() / b.num_items
        print(f"{name:12s} M={M:3d} gpu-f32 {g - f32:+.2e}  cpubf16-f32 {b16 - f32:+.2e}", flush=True)
