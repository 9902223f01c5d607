"""Pins the oracle's CLIP vision tower + head_dim-80 GPTNeoX (BASELINE C5's shapes:
CLIP-ViT-L/14-336 + Pythia-2.8B, scaled down) against the real HF modules run live in
this container (transformers' LlavaForConditionalGeneration(CLIPVisionConfig,
GPTNeoXConfig)): quick-GELU MLP, pre_layrnorm, bias-free patch conv with a
14-pixel patch (C·p·p = 588 -> the build's im2col pads K to 592), 20 rotary dims.
The HF modules are the reference's arithmetic for src/models/llava.py:23-58."""

import pytest
import torch

from oracle import model as O
from oracle.hf_mapping import build_to_hf

transformers = pytest.importorskip("transformers")


def _tiny():
    vc = O.VisionCfg(hidden=64, layers=3, heads=1, ffn=128, image=28, patch=14, eps=1e-5,
                     act="quick_gelu", pre_ln=True, patch_bias=False)
    tc = O.TextCfg(hidden=160, layers=2, heads=2, ffn=320, vocab=512)
    return O.MMCfg(vision=vc, text=tc, image_token_id=511)


def _hf(cfg):
    from transformers import (CLIPVisionConfig, GPTNeoXConfig, LlavaConfig,
                              LlavaForConditionalGeneration)

    v, t = cfg.vision, cfg.text
    vc = CLIPVisionConfig(hidden_size=v.hidden, num_hidden_layers=v.layers,
                          num_attention_heads=v.heads, intermediate_size=v.ffn, image_size=v.image,
                          patch_size=v.patch, hidden_act="quick_gelu", layer_norm_eps=v.eps)
    tc = GPTNeoXConfig(vocab_size=t.vocab, hidden_size=t.hidden, num_hidden_layers=t.layers,
                       num_attention_heads=t.heads, intermediate_size=t.ffn, rotary_pct=0.25,
                       rotary_emb_base=10000, max_position_embeddings=256,
                       use_parallel_residual=True, hidden_act="gelu", layer_norm_eps=1e-5,
                       tie_word_embeddings=False)
    lc = LlavaConfig(vision_config=vc, text_config=tc, image_token_id=cfg.image_token_id,
                     vision_feature_layer=-2, vision_feature_select_strategy="default",
                     projector_hidden_act="gelu")
    lc._attn_implementation = "sdpa"
    m = LlavaForConditionalGeneration(lc)
    return m


def test_clip_d80_oracle_matches_hf():
    torch.manual_seed(0)
    cfg = _tiny()
    assert cfg.text.head_dim == 80 and cfg.text.rot_dims == 20 and cfg.vision.patch_k == 592
    P = O.init_params(cfg, seed=0)
    assert torch.all(P["vision.patch.weight"][:, 588:] == 0)
    m = _hf(cfg)
    m.load_state_dict(build_to_hf(P, m.state_dict(), cfg.vision.used_layers, cfg.text.layers, True))
    batch = O.make_batch(cfg, 2, 45, seed=1)
    with torch.no_grad():
        hf32 = m(**batch).loss.item()
        with torch.autocast("cpu", dtype=torch.bfloat16):
            hf16 = m(**batch).loss.item()
        o32 = O.forward_loss(P, cfg, batch, "fp32").item()
        o16 = O.forward_loss(P, cfg, batch, "bf16").item()
    # the restatement performs HF's ops in HF's order: bit-equal in fp32 and bf16 autocast
    assert o32 == hf32, (o32, hf32)
    assert o16 == hf16, (o16, hf16)
