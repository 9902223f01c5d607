"""Full-size parity of the HIP step with HF goldens beyond the
forward loss: tests/golden/fullsize_r2.json and fullsize_r3.json, generated in the build
container by oracle/gen_golden.py generate_fullsize_r2() / oracle/gen_golden_r3.py (weights
oracle.init_params(seed=0), batches oracle.make_batch(seed=1); the oracle is bit-equal to the
HF modules on these models' forward, tests/golden/fullsize_losses.json and the
`oracle_loss_*` fields).

The bar for every quantity q is ABSOLUTE: |HIP − HF bf16| < 1e-4 + 2·σ_q, where σ_q is q's
own measured bf16 rounding noise — the std of the CPU bf16-autocast value over 1e-7 relative
weight perturbations (the fp32 value does not move), measured for the forward loss, the
step-1 gradient norm, every step loss and the loss after the steps.  Two valid bf16
implementations sit at that distance from each other.  A value within the same bar of the
HF fp32 result (the exact arithmetic) also passes (parity_record.within); both deltas are
recorded.  Every achieved delta is appended to
the parity record (tests/parity_record.py → profiles/<round>/parity_deltas.json).

* C5 CLIP-ViT-L/14-336 + Pythia-2.8B @ 576 + 511 tokens: forward loss at M = 2 and 16; the
  training scalars (M = 2, AdamW lr 1e-4, two steps) with the reference's C5 setting,
  ZeRO-3 + host offload (src/train.py:182-213), at world 1.
* C3 ViT-B/16 + Pythia-1B (M = 16 as two micro-batches of 8, AdamW) and C2 Pythia-1B @ 2049
  (M = 1, Adam betas (0.9, 0.95), clip 1.0): step-1 gradient L2 norm, the losses of two
  optimizer steps (lr 1e-4) and the loss after them.
* C4-shaped: the same C2 scalars with sharding="zero_3" and activation checkpointing on
  (world 1: the ZeRO-3 residency / per-unit reduce / recompute machinery in the loop).
* llava-pretrain, the reference's own model (src/models/llava.py:22-58: CLIP-ViT-L/14-336 +
  Llama-3.2-1B, tower and LLM frozen): forward loss at M = 2 and 16; projector gradient norm,
  two AdamW steps (lr 1e-3) and the loss after them at M = 16 (two micro-batches of 8).
"""

import json
import os

import pytest
import torch

from oracle import model as O
from parity_record import bar, record

pytestmark = pytest.mark.gpu

_G = os.path.join(os.path.dirname(__file__), "golden")
GOLD = json.load(open(os.path.join(_G, "fullsize_r2.json")))
GOLD3 = json.load(open(os.path.join(_G, "fullsize_r3.json")))
try:  # round 4: C3 at the bench micro-batch, sigma re-measured with >= 12 perturbations
    GOLD4 = json.load(open(os.path.join(_G, "fullsize_r4.json")))
except OSError:
    GOLD4 = {}
try:  # round 5: C2 at M = 16 (oracle/gen_golden_r5.py)
    GOLD5 = json.load(open(os.path.join(_G, "fullsize_r5.json")))
except OSError:
    GOLD5 = {}
try:  # round 6: llava-pretrain projector training at M = 32 (oracle/gen_golden_r6.py)
    GOLD6 = json.load(open(os.path.join(_G, "fullsize_r6.json")))
except OSError:
    GOLD6 = {}


def _noise(key, r3_noise):
    """The round-4 sigma of a round-3 record when re-measured (more perturbations)."""
    rec = GOLD4.get("sigma12", {}).get(key)
    return rec if rec is not None else r3_noise


def _ocfg(name):
    from test_parity_gpu import oracle_cfg

    from multimodal_llm_pretraining_amd import config as C

    return oracle_cfg(C.get_config(name))


def _forward_loss(name, M):
    from multimodal_llm_pretraining_amd import config as C
    from multimodal_llm_pretraining_amd.engine import Batch, Engine
    from multimodal_llm_pretraining_amd.params import ParamStore

    ocfg = _ocfg(name)
    P = O.init_params(ocfg, seed=0)
    batch = O.make_batch(ocfg, M, 511, seed=1)
    cfg = C.get_config(name)
    store = ParamStore(C.param_shapes(cfg), "cuda")
    store.load(P)
    del P
    store.refresh_shadow()
    eng = Engine(cfg, store)
    b = Batch(cfg, batch["input_ids"], batch["labels"], batch["pixel_values"], store.device)
    return eng.forward(b, 1.0 / b.num_items, need_grad=False).item() / b.num_items


@pytest.mark.parametrize("key,M", [("clip-l14-336-pythia-2.8b", 2), ("clip-l14-336-pythia-2.8b-M16", 16)])
def test_c5_full_size_loss(key, M):
    gold = GOLD[key]
    loss = _forward_loss("clip-l14-336-pythia-2.8b", M)
    ref, tol = gold["loss_bf16_autocast"], bar(gold["bf16_noise_std"])
    assert record(f"c5_loss[{key}]", "loss", loss, ref, tol, sigma=gold["bf16_noise_std"],
                  fp32=gold["loss_fp32"]), (loss, ref)


@pytest.mark.parametrize("key,M", [("llava-pretrain", 2), ("llava-pretrain-M16", 16)])
def test_llava_pretrain_full_size_loss(key, M):
    gold = GOLD3[key]
    # the oracle restates HF's LlavaForConditionalGeneration(CLIP, Llama) bit for bit here
    assert gold["oracle_loss_bf16_autocast"] == gold["loss_bf16_autocast"]
    loss = _forward_loss("llava-pretrain", M)
    noise = _noise(key, gold)  # M = 2: re-measured over 16 perturbations
    sigma = noise["bf16_noise_std"]
    smp = noise.get("samples")
    ref, tol = gold["loss_bf16_autocast"], bar(sigma)
    assert record(f"llava_pretrain_loss[{key}]", "loss", loss, ref, tol, sigma=sigma,
                  fp32=gold["loss_fp32"], noise_mean=sum(smp) / len(smp) if smp else None), (loss, ref)


def _train_scalars(name, gold, micro, text_len, sharding="", ac=False, offload=False):
    from multimodal_llm_pretraining_amd import kernels as K
    from multimodal_llm_pretraining_amd.optim import AdamConfig
    from multimodal_llm_pretraining_amd.trainer import ManualTrainer, StepConfig

    ocfg = _ocfg(name)
    P = O.init_params(ocfg, seed=0)
    full = O.make_batch(ocfg, micro[0] * micro[1], text_len, seed=1)
    n = micro[1]
    parts = [{k: v[i * n:(i + 1) * n] for k, v in full.items()} for i in range(micro[0])]
    adam = AdamConfig(lr=gold["lrs"][0], betas=tuple(gold["betas"]), eps=1e-8, weight_decay=0.0,
                      adamw=gold["optimizer"] == "AdamW", max_grad_norm=gold["clip"])
    tr = ManualTrainer(StepConfig(model=name, scheduler="constant", sharding=sharding,
                                  activation_checkpointing=ac, offload=offload), adam, "cuda",
                       init=False)
    tr.store.load(P)
    del P
    tr.store.refresh_shadow()
    tr.store.refresh_transposed()  # (an offload's host master is taken at its first step)
    batches = [tr.stage(p) for p in parts]
    n_items = sum(b.num_items for b in batches)
    losses, gnorm = [], None
    for step in range(2):
        tot = 0.0
        for i, b in enumerate(batches):
            tot += tr.manual_training_step(b, n_items, i == len(batches) - 1).item()
        if step == 0:
            if tr.mode == "zero3":
                # the last units' shard reductions run on the comm stream (manual_optimization_
                # step joins it in reduce_grads before its clip norm; world 1 here, so the join
                # alone is that call's effect)
                torch.cuda.current_stream().wait_stream(tr.sync.stream)
            ss = tr.sync.global_sumsq(K) if tr.mode == "zero3" else tr.opt.grad_sumsq()
            gnorm = ss.item() ** 0.5
        tr.manual_optimization_step()
        losses.append(tot / n_items)
    tr.flush()
    after = sum(tr.engine.forward(b, 1.0 / n_items, need_grad=False).item() for b in batches) / n_items
    return {"grad_norm": gnorm, "losses": losses, "loss_after": after}


def _noise_mean(noise, what):
    """Mean of quantity `what` over the noise samples (the unperturbed bf16 run + the weight
    perturbations) when the golden keeps them: recorded beside each delta (a single HF bf16
    run is one draw of that distribution; the C5 gradient norm's unperturbed run sits 2.1
    sigma below its mean, HIP's at +0.02 sigma)."""
    smp = noise.get("samples") if isinstance(noise, dict) else None
    if not smp:
        return None
    def q(x):
        return x["grad_norm"] if what == "grad_norm" else (
            x["loss_after"] if what == "loss_after" else x["losses"][int(what[4:])])
    return sum(q(x) for x in smp) / len(smp)


def _check(test, got, gold, noise):
    """Every training scalar within 1e-4 + 2 sigma_q of the HF bf16 value (or of the HF fp32
    value, parity_record.within), absolute."""
    bf, f32 = gold["bf16"], gold["fp32"]
    rows = [("grad_norm", got["grad_norm"], bf["grad_norm"], f32["grad_norm"], noise["grad_norm"])]
    rows += [(f"loss{i}", g, b, f, s) for i, (g, b, f, s) in
             enumerate(zip(got["losses"], bf["losses"], f32["losses"], noise["losses"]))]
    rows.append(("loss_after", got["loss_after"], bf["loss_after"], f32["loss_after"],
                 noise["loss_after"]))
    bad = []
    for what, g, b, f, s in rows:
        if not record(test, what, g, b, bar(s), sigma=s, fp32=f,
                      noise_mean=_noise_mean(noise, what)):
            bad.append((what, g, b, f, s))
    assert not bad, bad


def test_c3_full_size_grad_norm_and_two_steps():
    got = _train_scalars("vit-b16-pythia-1b", GOLD["c3train"], (2, 8), 511)
    _check("c3_train", got, GOLD["c3train"], GOLD3["c3train_noise"])


def test_c2_full_size_grad_norm_and_two_steps():
    got = _train_scalars("pythia-1b", GOLD["c2train"], (1, 1), 2049)
    _check("c2_train", got, GOLD["c2train"], GOLD3["c2train_noise"])


@pytest.mark.skipif(len(GOLD5.get("c2train-M16", {}).get("noise", {}).get("samples", [])) < 8,
                    reason="round-5 C2 M = 16 golden not generated")
def test_c2_full_size_M16_grad_norm_and_two_steps():
    """C2 (Pythia-1B @ 2049, Adam betas (0.9, 0.95), clip 1.0) at M = 16 (8 accumulated
    micro-batches of 2): the M = 1 record's sigma (6.3e-4 on the loss after two steps) would
    hide a 1e-3 optimizer-path regression; at M = 16 the step losses' sigma is 4x smaller
    (VERDICT r04 #6)."""
    gold = GOLD5["c2train-M16"]
    got = _train_scalars("pythia-1b", gold, (8, 2), 2049)
    _check("c2_train_M16", got, gold, gold["noise"])


def test_c4_shaped_zero3_ac_grad_norm_and_two_steps():
    got = _train_scalars("pythia-1b", GOLD["c2train"], (1, 1), 2049, sharding="zero_3", ac=True)
    _check("c4_shaped_zero3_ac_train", got, GOLD["c2train"], GOLD3["c2train_noise"])


def test_c5_full_size_zero3_offload_grad_norm_and_two_steps():
    """BASELINE C5 as configured: CLIP-L/14-336 + Pythia-2.8B with ZeRO-3 + host offload
    (the fp32 master and Adam moments in pinned host memory, CPU Adam) at world 1."""
    gold = GOLD3["c5train"]
    got = _train_scalars("clip-l14-336-pythia-2.8b", gold, (1, 2), 511, sharding="zero_3",
                         offload=True)
    _check("c5_zero3_offload_train", got, gold, _noise("c5train", gold["noise"]))


@pytest.mark.skipif(len(GOLD6.get("c5train-M8", {}).get("noise", {}).get("samples", [])) < 8,
                    reason="round-6 C5 M = 8 golden not generated")
def test_c5_full_size_M8_zero3_offload_grad_norm_and_two_steps():
    """C5 (CLIP-L/14-336 + Pythia-2.8B, ZeRO-3 + host offload at world 1) at M = 8 as 4
    accumulated micro-batches of 2: round 3's M = 2 record (7 noise samples) left the grad norm
    at 0.97 of its bf16 bar (C5 at M >= 8); sigma shrinks with M."""
    gold = GOLD6["c5train-M8"]
    got = _train_scalars("clip-l14-336-pythia-2.8b", gold, (4, 2), 511, sharding="zero_3",
                         offload=True)
    _check("c5_zero3_offload_train_M8", got, gold, gold["noise"])


def test_llava_pretrain_full_size_projector_train():
    """llava-pretrain (tower + LLM frozen, src/models/llava.py:49-52): the projector's
    gradient norm and two AdamW steps at the recipe's lr 1e-3, M = 16 as 2 x 8."""
    gold = GOLD3["llava-pretrain-train"]
    got = _train_scalars("llava-pretrain", gold, (2, 8), 511)
    _check("llava_pretrain_train", got, gold, _noise("llava-pretrain-train", gold["noise"]))


@pytest.mark.skipif(len(GOLD6.get("llava-pretrain-train-M32", {}).get("noise", {})
                        .get("samples", [])) < 8, reason="round-6 llava M = 32 golden not generated")
def test_llava_pretrain_full_size_projector_train_M32():
    """The same projector training at M = 32 (4 accumulated micro-batches of 8): the M = 16
    record's sigma (3.6e-4 on the step-1 loss) let the single HF bf16 draw sit 1.1 bars from the
    HIP value; sigma shrinks with M."""
    gold = GOLD6["llava-pretrain-train-M32"]
    got = _train_scalars("llava-pretrain", gold, (4, 8), 511)
    _check("llava_pretrain_train_M32", got, gold, gold["noise"])


@pytest.mark.skipif("c3train-M64" not in GOLD4, reason="round-4 golden not generated")
def test_c3_bench_micro_batch_step0_loss_bare_bar():
    """C3 at the bench's own micro-batch, M = 64 (8 accumulated micro-batches of 8, AdamW lr
    1e-4): step-1 gradient norm, two step losses and the loss after them against HF bf16 (or
    fp32).  The step-0 loss — the north star's "loss on a fixed synthetic
    image-text batch" — is held to the BARE 1e-4, no noise allowance; every
    quantity whose measured sigma is >= 5e-5 (the step-1 loss, gradient norm and loss after
    two updates at M = 64) keeps 1e-4 + 2 sigma.  The sigma is recorded beside each delta."""
    gold = GOLD4["c3train-M64"]
    got = _train_scalars("vit-b16-pythia-1b", gold, (8, 8), 511)
    noise = gold.get("noise")
    bf, f32 = gold["bf16"], gold["fp32"]
    rows = [("grad_norm", got["grad_norm"], bf["grad_norm"], f32["grad_norm"],
             noise and noise["grad_norm"])]
    rows += [(f"loss{i}", g, b, f, noise and noise["losses"][i]) for i, (g, b, f) in
             enumerate(zip(got["losses"], bf["losses"], f32["losses"]))]
    rows.append(("loss_after", got["loss_after"], bf["loss_after"], f32["loss_after"],
                 noise and noise["loss_after"]))
    # The bare bar for every quantity whose bf16 noise (sigma over the weight perturbations)
    # lies below half of it: the step-0 loss (the north-star quantity: the loss of a fixed
    # synthetic batch) and the step-1 loss.  The step-1 gradient norm and the loss after two
    # updates carry sigma ~1.1e-4 at M = 64 (13 perturbations, tests/golden/fullsize_r4.json):
    # HF's own bf16 run moves by more than 1e-4 under a 1e-7-relative weight perturbation, so
    # those two are held to 1e-4 + 2 sigma like the M = 16 records.
    def bar_of(s):
        return 1e-4 if s is None or s < 5e-5 else 1e-4 + 2 * s
    bad = [r for r in rows if not record("c3_train_M64_bare", r[0], r[1], r[2], bar_of(r[4]),
                                         sigma=r[4], fp32=r[3],
                                         noise_mean=_noise_mean(gold.get("noise"), r[0]))]
    assert not bad, bad
