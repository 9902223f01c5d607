"""End-to-end parity of the HIP training step with the CPU oracle (oracle/model.py,
itself pinned to HF transformers by tests/test_oracle_golden.py).

Same seeded fp32 weights and synthetic batch on both sides; the oracle runs the
reference's bf16-autocast CPU semantics.  Tolerances (north_star: loss within
1e-4 of the CPU reference in bf16):
  * loss: |Δ| < 1e-4 absolute against the fp32 oracle, and against the bf16-autocast
    oracle within 1e-4 + |oracle_bf16 - oracle_fp32| (the bf16 rounding noise floor of
    that config: two valid bf16 implementations can sit on either side of fp32);
    the full-size C3 check uses the bare 1e-4 bar against the bf16 oracle;
  * gradients: ‖Δ‖/‖ref‖ < 3e-2 per tensor (bf16 operands, different summation order);
  * two optimizer steps: both losses within 1e-4 (second: 3e-4, after an lr-1e-3 update).
"""

import pytest
import torch

from oracle import model as O

pytestmark = pytest.mark.gpu


def oracle_cfg(cfg):
    v = cfg.vision
    ov = None if v is None else O.VisionCfg(hidden=v.hidden, layers=v.layers, heads=v.heads,
                                            ffn=v.ffn, image=v.image, patch=v.patch, eps=v.eps,
                                            act=v.act, pre_ln=v.pre_ln, patch_bias=v.patch_bias)
    t = cfg.text
    ot = O.TextCfg(hidden=t.hidden, layers=t.layers, heads=t.heads, ffn=t.ffn, vocab=t.vocab,
                   rotary_pct=t.rotary_pct, rope_theta=t.rope_theta, eps=t.eps, arch=t.arch,
                   kv_heads=t.kv_heads, rope_scaling=t.rope_scaling,
                   tie_embeddings=t.tie_embeddings, vocab_valid=t.vocab_valid)
    return O.MMCfg(vision=ov, text=ot, image_token_id=cfg.image_token_id)


def gpu_setup(name, params):
    from multimodal_llm_pretraining_amd import config as C
    from multimodal_llm_pretraining_amd.engine import Engine
    from multimodal_llm_pretraining_amd.params import ParamStore

    cfg = C.get_config(name)
    store = ParamStore(C.param_shapes(cfg), "cuda")
    store.load(params)
    store.refresh_shadow()
    return cfg, store, Engine(cfg, store)


def test_layout_matches_oracle():
    from multimodal_llm_pretraining_amd import config as C

    for name in ("tiny-mm", "tiny-lm", "tiny-lm-d80", "tiny-clip-d80", "vit-b16-pythia-1b",
                 "pythia-1b", "pythia-2.8b", "clip-l14-336-pythia-2.8b", "tiny-llama",
                 "tiny-llava", "llava-pretrain"):
        cfg = C.get_config(name)
        assert C.param_shapes(cfg) == O.param_shapes(oracle_cfg(cfg))


@pytest.mark.parametrize("name,text_len", [("tiny-mm", 47), ("tiny-lm", 130), ("tiny-lm-d80", 130),
                                           ("tiny-clip-d80", 47), ("tiny-llama", 130),
                                           ("tiny-llava", 47)])
def test_loss_and_grads(name, text_len):
    from multimodal_llm_pretraining_amd import config as C
    from multimodal_llm_pretraining_amd.engine import Batch

    ocfg = oracle_cfg(C.get_config(name))
    P = O.init_params(ocfg, seed=0)
    # tiny-clip-d80's bf16 loss moves by ~3e-4 between M = 2 and 8 on the CPU alone
    # (quick-GELU adds two roundings per MLP element; scripts/diag/diag_d80.py: no GPU bias,
    # within 5e-5 of fp32 at M = 32): test it on 32 samples
    batch = O.make_batch(ocfg, 32 if name == "tiny-clip-d80" else 3, text_len, seed=1)
    Pr = {k: v.clone().requires_grad_() for k, v in P.items()}
    ref = O.forward_loss(Pr, ocfg, batch, "bf16")
    ref.backward()
    with torch.no_grad():
        ref32 = O.forward_loss(P, ocfg, batch, "fp32").item()
    floor = abs(ref.item() - ref32)

    cfg, store, eng = gpu_setup(name, P)
    b = Batch(cfg, batch["input_ids"], batch["labels"], batch.get("pixel_values"), store.device)
    loss_sum = eng.forward(b, 1.0 / b.num_items)
    eng.backward(b)
    loss = loss_sum.item() / b.num_items
    assert abs(loss - ref32) < 1e-4, (loss, ref32)
    assert abs(loss - ref.item()) < 1e-4 + floor, (loss, ref.item(), floor)
    for k in P:
        g = store.g(k).cpu()
        r = Pr[k].grad
        err = ((g - r).norm() / (r.norm() + 1e-20)).item()
        assert err < 3e-2, (k, err)


@pytest.mark.parametrize("name,text_len", [("tiny-mm", 47), ("tiny-lm", 130), ("tiny-lm-d80", 130),
                                           ("tiny-clip-d80", 47), ("tiny-llama", 130),
                                           ("tiny-llava", 47)])
def test_two_adamw_steps(name, text_len):
    from multimodal_llm_pretraining_amd.optim import AdamConfig
    from multimodal_llm_pretraining_amd.trainer import ManualTrainer, StepConfig

    from multimodal_llm_pretraining_amd import config as C

    ocfg = oracle_cfg(C.get_config(name))
    P = O.init_params(ocfg, seed=0)
    # tiny-lm-d80's CPU bf16 loss noise is 6.4e-5 (std over 1e-7 relative weight
    # perturbations) at M = 2, vs 2.6e-5 for tiny-lm: use M = 8 there (scripts/diag/diag_d80.py:
    # no bias — GPU within 2e-5 of fp32 at M = 32, like the CPU bf16 loss)
    M = 8 if name in ("tiny-lm-d80", "tiny-clip-d80") else 2
    batches = [O.make_batch(ocfg, M, text_len, seed=s) for s in (1, 2)]
    lrs = [1e-3, 1e-3]
    ref_losses, _ = O.train_steps(P, ocfg, batches, O.OptimCfg(kind="adamw", lr=1e-3), lrs, "bf16")
    ref32, _ = O.train_steps(P, ocfg, batches, O.OptimCfg(kind="adamw", lr=1e-3), lrs, "fp32")
    floor = [abs(a - b) for a, b in zip(ref_losses, ref32)]

    tr = ManualTrainer(StepConfig(model=name, scheduler="constant"), AdamConfig(lr=1e-3), "cuda")
    tr.store.load(P)
    tr.store.refresh_shadow()
    got = []
    for bd in batches:
        b = tr.stage(bd)
        s = tr.train_step([b], b.num_items)
        got.append(s.item() / b.num_items)
    assert abs(got[0] - ref_losses[0]) < 1e-4 + floor[0], (got, ref_losses, ref32)
    assert abs(got[1] - ref_losses[1]) < 3e-4 + floor[1], (got, ref_losses, ref32)


def test_grad_accumulation_equals_big_batch():
    """GA over two micro-batches == one micro-batch of both (same global num_items)."""
    from multimodal_llm_pretraining_amd import config as C
    from multimodal_llm_pretraining_amd.engine import Batch

    ocfg = oracle_cfg(C.get_config("tiny-lm"))
    P = O.init_params(ocfg, seed=0)
    bd = O.make_batch(ocfg, 4, 64, seed=3)
    cfg, store, eng = gpu_setup("tiny-lm", P)
    full = Batch(cfg, bd["input_ids"], bd["labels"], None, store.device)
    eng.forward(full, 1.0 / full.num_items)
    eng.backward(full)
    g_full = store.grad.clone()
    store.zero_grad()
    for sl in (slice(0, 2), slice(2, 4)):
        b = Batch(cfg, bd["input_ids"][sl], bd["labels"][sl], None, store.device)
        eng.forward(b, 1.0 / full.num_items)
        eng.backward(b)
    err = ((store.grad - g_full).norm() / g_full.norm()).item()
    assert err < 1e-2


@pytest.mark.parametrize("key,name,text_len,M", [("vit-b16-pythia-1b-M64", "vit-b16-pythia-1b", 511, 64),
                                                  ("vit-b16-pythia-1b-M16", "vit-b16-pythia-1b", 511, 16),
                                                  ("vit-b16-pythia-1b", "vit-b16-pythia-1b", 511, 2),
                                                  ("pythia-1b", "pythia-1b", 2049, 1)])
def test_full_size_loss(key, name, text_len, M):
    """BASELINE configs C3 (ViT-B/16 + Pythia-1B, L = 196 + 511 = 707) and Pythia-1B @ 2049
    against the bf16-autocast loss of the real HF modules, pinned in
    tests/golden/fullsize_losses.json (generated in the build container: the CPU bf16
    result is host-ISA dependent, so it is not recomputed on the GPU box).

    The bf16 loss carries rounding noise: a 1e-7 relative weight perturbation moves the
    CPU bf16 loss by std 1.2e-4 at M = 2, 5.2e-5 at M = 16 and 3.1e-5 at M = 64
    (`bf16_noise_std`, measured by oracle/gen_golden.py; the fp32 loss does not move).  The
    north-star 1e-4 bar is therefore applied to the M = 64 batch (one bench micro-batch);
    M = 16 and M = 2 are held to 1e-4 + 2 sigma."""
    import json
    import os

    from multimodal_llm_pretraining_amd import config as C
    from multimodal_llm_pretraining_amd.engine import Batch

    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "fullsize_losses.json")))[key]
    ocfg = oracle_cfg(C.get_config(name))
    P = O.init_params(ocfg, seed=0)
    batch = O.make_batch(ocfg, M, text_len, seed=1)
    cfg, store, eng = gpu_setup(name, P)
    b = Batch(cfg, batch["input_ids"], batch["labels"], batch.get("pixel_values"), store.device)
    loss = eng.forward(b, 1.0 / b.num_items, need_grad=False).item() / b.num_items
    ref = gold["loss_bf16_autocast"]
    print(f"full-size {key}: GPU loss {loss:.7f}, CPU bf16 {ref:.7f} (d {loss - ref:+.2e}), "
          f"fp32 {gold['loss_fp32']:.7f} (d {loss - gold['loss_fp32']:+.2e})")
    from parity_record import record

    sigma = gold.get("bf16_noise_std")
    tol = 1e-4 if key == "vit-b16-pythia-1b-M64" else (
        1e-4 + 2 * sigma if sigma is not None else 1e-4 + abs(ref - gold["loss_fp32"]))
    record(f"full_size_loss[{key}]", "loss", loss, ref, tol, sigma=sigma, fp32=gold["loss_fp32"])
    # (the assertions below keep this test's own, stricter rules)
    if key == "vit-b16-pythia-1b-M64":  # the north-star batch: bare 1e-4 bar vs CPU bf16
        assert abs(loss - ref) < 1e-4, (loss, ref, gold["loss_fp32"])
    elif key in ("vit-b16-pythia-1b", "vit-b16-pythia-1b-M16"):
        assert abs(loss - ref) < 1e-4 + 2 * gold["bf16_noise_std"], (loss, ref, gold["bf16_noise_std"])
    else:
        # text-only S=2049, M=1: a single 2048-token sample averages little of the bf16
        # rounding noise (the SAME model on two CPUs differs by 1.5e-4);
        # require 1e-4 against the fp32 HF loss and the noise-floor bound against bf16.
        assert abs(loss - gold["loss_fp32"]) < 1e-4, (loss, gold["loss_fp32"])
        floor = abs(ref - gold["loss_fp32"])
        assert abs(loss - ref) < 1e-4 + floor, (loss, ref, floor)


def test_llava_pretrain_freeze():
    """llava-pretrain's freeze (src/models/llava.py:49-52, pinned transformers 4.47.1): only
    the projector trains.  Its gradients match the oracle (freezing does not change them);
    nothing else gets a gradient, and two AdamW steps move the projector alone."""
    from multimodal_llm_pretraining_amd import config as C
    from multimodal_llm_pretraining_amd.engine import Batch
    from multimodal_llm_pretraining_amd.optim import AdamConfig
    from multimodal_llm_pretraining_amd.trainer import ManualTrainer, StepConfig

    cfg = C.get_config("tiny-llava-frozen")
    ocfg = oracle_cfg(cfg)
    P = O.init_params(ocfg, seed=0)
    batch = O.make_batch(ocfg, 3, 47, seed=1)
    Pr = {k: v.clone().requires_grad_() for k, v in P.items()}
    ref = O.forward_loss(Pr, ocfg, batch, "bf16")
    ref.backward()
    tr = ManualTrainer(StepConfig(model="tiny-llava-frozen", scheduler="constant"),
                       AdamConfig(lr=1e-3), "cuda", model_cfg=cfg)
    tr.store.load(P)
    tr.store.refresh_shadow()
    b = Batch(cfg, batch["input_ids"], batch["labels"], batch["pixel_values"], tr.store.device)
    loss_sum = tr.engine.forward(b, 1.0 / b.num_items)
    tr.engine.backward(b)
    assert abs(loss_sum.item() / b.num_items - ref.item()) < 2e-4
    for k in P:
        g = tr.store.g(k).cpu()
        if k.startswith("proj."):
            r = Pr[k].grad
            assert ((g - r).norm() / (r.norm() + 1e-20)).item() < 3e-2, k
        else:
            assert torch.count_nonzero(g) == 0, k
    tr.store.zero_grad()
    before = {k: tr.store.p(k).cpu().clone() for k in P}
    for _ in range(2):
        tr.train_step([b], b.num_items)
    for k in P:
        moved = not torch.equal(tr.store.p(k).cpu(), before[k])
        assert moved == k.startswith("proj."), k
