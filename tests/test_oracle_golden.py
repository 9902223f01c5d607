"""Pins the CPU oracle (oracle/model.py) to golden vectors produced by the real HF
transformers modules that hold the reference's arithmetic (oracle/gen_golden.py):
losses (fp32 and bf16 autocast), every fp32 gradient, and parameters after two
AdamW steps.  CPU only."""

import json
import os

import pytest
import torch
from safetensors.torch import load_file

from oracle import model as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")

CFGS = {
    "tiny_llava_vit_gptneox": O.MMCfg(
        vision=O.VisionCfg(hidden=64, layers=3, heads=4, ffn=128, image=32, patch=16),
        text=O.TextCfg(hidden=64, layers=2, heads=4, ffn=256, vocab=512),
        image_token_id=511),
    "tiny_pythia": O.MMCfg(vision=None, text=O.TextCfg(hidden=64, layers=2, heads=2, ffn=256, vocab=256)),
}


def _load(name):
    t = load_file(os.path.join(GOLD, f"{name}.safetensors"))
    with open(os.path.join(GOLD, f"{name}.json")) as f:
        meta = json.load(f)
    pre = lambda p: {k[len(p):]: v for k, v in t.items() if k.startswith(p)}  # noqa: E731
    return pre("w."), pre("g."), pre("a."), pre("b."), meta


@pytest.mark.parametrize("name", list(CFGS))
def test_layout_matches_fixture(name):
    w, *_ = _load(name)
    shapes = O.param_shapes(CFGS[name])
    assert set(shapes) == set(w)
    for k, s in shapes.items():
        assert tuple(w[k].shape) == s, k


@pytest.mark.parametrize("name", list(CFGS))
def test_oracle_losses(name):
    w, _, _, b, meta = _load(name)
    cfg = CFGS[name]
    l32 = O.forward_loss(w, cfg, b, "fp32").item()
    l16 = O.forward_loss(w, cfg, b, "bf16").item()
    assert abs(l32 - meta["loss_fp32"]) < 2e-6
    assert abs(l16 - meta["loss_bf16_autocast"]) < 2e-5


@pytest.mark.parametrize("name", list(CFGS))
def test_oracle_grads(name):
    w, g, _, b, _ = _load(name)
    cfg = CFGS[name]
    P = {k: v.clone().requires_grad_() for k, v in w.items()}
    O.forward_loss(P, cfg, b, "fp32").backward()
    for k, ref in g.items():
        got = P[k].grad
        err = (got - ref).abs().max().item()
        assert err <= 1e-6 + 1e-4 * ref.abs().max().item(), (k, err)


@pytest.mark.parametrize("name", list(CFGS))
def test_oracle_two_adamw_steps(name):
    w, _, a, b, meta = _load(name)
    cfg = CFGS[name]
    opt = O.OptimCfg(kind="adamw", lr=meta["lrs"][0], betas=tuple(meta["betas"]), eps=meta["eps"],
                     weight_decay=meta["weight_decay"])
    losses, after = O.train_steps(w, cfg, [b, b], opt, meta["lrs"], precision="fp32")
    assert abs(losses[0] - meta["train_losses"][0]) < 2e-6
    assert abs(losses[1] - meta["train_losses"][1]) < 2e-5
    for k, ref in a.items():
        assert (after[k] - ref).abs().max().item() < 2e-5, k


def test_flops_matches_survey():
    # ViT-B/16 + Pythia-1B @ 707 = 4.169 TFLOP/sample; Pythia-1B@2049 = 12.818
    mm = O.MMCfg(vision=O.VisionCfg(), text=O.TextCfg())
    assert abs(O.flops_per_sample(mm, 511) / 1e12 - 4.169) < 0.01
    lm = O.MMCfg(vision=None, text=O.TextCfg())
    assert abs(O.flops_per_sample(lm, 2049) / 1e12 - 12.818) < 0.01


def test_batch_semantics():
    cfg = O.MMCfg(vision=O.VisionCfg(), text=O.TextCfg())
    b = O.make_batch(cfg, 2, 511)
    assert b["input_ids"].shape == (2, 707)
    assert (b["input_ids"][:, :196] == 50303).all() and (b["input_ids"][:, 196:] < 50303).all()
    assert (b["labels"][:, :196] == -100).all()
    assert b["pixel_values"].shape == (2, 3, 224, 224)
    assert torch.equal(b["attention_mask"], torch.ones_like(b["input_ids"]))


@pytest.mark.parametrize("cls,wd", [("AdamW", 0.0), ("AdamW", 0.1), ("Adam", 0.0), ("Adam", 0.05)])
def test_golden_adam_restatement_is_torch(cls, wd):
    """oracle/gen_golden_r3.adam_step_ (the memory-lean optimizer of the full-size goldens)
    is bit-identical to torch.optim.Adam / AdamW (foreach=False) over three steps."""
    from oracle.gen_golden_r3 import adam_step_

    g = torch.Generator().manual_seed(3)
    p0 = torch.randn(1000, generator=g)
    grads = [torch.randn(1000, generator=g) * 10 ** (-k) for k in range(3)]
    ref = p0.clone().requires_grad_()
    opt = getattr(torch.optim, cls)([ref], lr=1e-3, betas=(0.9, 0.95), eps=1e-8,
                                    weight_decay=wd, foreach=False)
    p, m, v = p0.clone(), torch.zeros(1000), torch.zeros(1000)
    for i, gr in enumerate(grads):
        ref.grad = gr.clone()
        opt.step()
        adam_step_(p, gr.clone(), m, v, i + 1, 1e-3, (0.9, 0.95), 1e-8, wd, cls == "AdamW")
        assert torch.equal(p, ref.detach()), (cls, wd, i)
