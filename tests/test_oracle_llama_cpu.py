"""Pins the oracle's Llama-3 text model (RMSNorm, GQA through SDPA enable_gqa, llama3-scaled RoPE,
SwiGLU, tied embeddings, padded vocabulary) and the reference's own llava-pretrain
composition (CLIP vision tower + projector + Llama, src/models/llava.py:22-58) against the
real HF modules run live in this container (transformers LlamaForCausalLM /
LlavaForConditionalGeneration(CLIPVisionConfig, LlamaConfig)), scaled down; loss and every
gradient.  The build's fused weights (q|k|v rows, blocked gate|up rows) map onto HF's
separate projections through oracle/hf_mapping.py."""

import pytest
import torch

from oracle import model as O
from oracle.hf_mapping import build_to_hf_llama

transformers = pytest.importorskip("transformers")

ROPE = (32.0, 1.0, 4.0, 64)  # llama3 scaling with a small original context: every band hit


def _text(kv=1):
    return O.TextCfg(hidden=256, layers=2, heads=4, ffn=256, vocab=520, vocab_valid=515,
                     rotary_pct=1.0, rope_theta=500000.0, eps=1e-5, arch="llama", kv_heads=kv,
                     rope_scaling=ROPE, tie_embeddings=True)


def _hf_llama_cfg(t):
    from transformers import LlamaConfig

    return LlamaConfig(vocab_size=t.n_vocab, hidden_size=t.hidden, intermediate_size=t.ffn,
                       num_hidden_layers=t.layers, num_attention_heads=t.heads,
                       num_key_value_heads=t.n_kv, hidden_act="silu", max_position_embeddings=256,
                       rms_norm_eps=t.eps, tie_word_embeddings=True,
                       rope_parameters={"rope_type": "llama3", "rope_theta": t.rope_theta,
                                        "factor": ROPE[0], "low_freq_factor": ROPE[1],
                                        "high_freq_factor": ROPE[2],
                                        "original_max_position_embeddings": ROPE[3]})


def _grads_match(P, cfg, batch, hf_model, to_hf):
    Pr = {k: v.clone().requires_grad_() for k, v in P.items()}
    O.forward_loss(Pr, cfg, batch, "fp32").backward()
    hf_model.zero_grad()
    hf_model(**batch).loss.backward()
    hf_g = {n: p.grad for n, p in hf_model.named_parameters() if p.grad is not None}
    mapped = to_hf({k: v.grad for k, v in Pr.items()})
    for n, g in hf_g.items():
        ref = mapped[n]
        # (+1e-6: the attention key biases have an analytically zero gradient)
        err = ((g - ref).norm() / (ref.norm() + 1e-6)).item()
        assert err < 1e-5, (n, err)


def test_llama_oracle_matches_hf():
    from transformers import LlamaForCausalLM

    torch.manual_seed(0)
    t = _text(kv=1)
    cfg = O.MMCfg(vision=None, text=t)
    P = O.init_params(cfg, seed=0)
    m = LlamaForCausalLM(_hf_llama_cfg(t))
    m.config._attn_implementation = "sdpa"
    m.load_state_dict(build_to_hf_llama(P, m.state_dict(), t, None))
    assert m.lm_head.weight.data_ptr() == m.model.embed_tokens.weight.data_ptr()  # tied
    batch = O.make_batch(cfg, 2, 96, seed=1)
    assert int(batch["input_ids"].max()) < t.n_vocab
    with torch.no_grad():
        hf32 = m(**batch).loss.item()
        with torch.autocast("cpu", dtype=torch.bfloat16):
            hf16 = m(**batch).loss.item()
        o32 = O.forward_loss(P, cfg, batch, "fp32").item()
        o16 = O.forward_loss(P, cfg, batch, "bf16").item()
    assert abs(o32 - hf32) < 2e-6, (o32, hf32)
    assert abs(o16 - hf16) < 2e-6, (o16, hf16)
    # a zero-init padded vocabulary row changes nothing: it is dropped before the loss
    _grads_match(P, cfg, batch, m, lambda G: build_to_hf_llama(G, dict(m.state_dict()), t, None))


def test_llava_clip_llama_oracle_matches_hf():
    from transformers import CLIPVisionConfig, LlavaConfig, LlavaForConditionalGeneration

    torch.manual_seed(0)
    t = _text(kv=2)
    t = O.TextCfg(**{**t.__dict__, "vocab": 1032, "vocab_valid": 1025})
    vc = O.VisionCfg(hidden=128, layers=3, heads=2, ffn=256, image=56, patch=14, eps=1e-5,
                     act="quick_gelu", pre_ln=True, patch_bias=False)
    cfg = O.MMCfg(vision=vc, text=t, image_token_id=1024)
    P = O.init_params(cfg, seed=0)
    lc = LlavaConfig(vision_config=CLIPVisionConfig(hidden_size=128, num_hidden_layers=3,
                                                    num_attention_heads=2, intermediate_size=256,
                                                    image_size=56, patch_size=14,
                                                    hidden_act="quick_gelu", layer_norm_eps=1e-5),
                     text_config=_hf_llama_cfg(t), image_token_id=1024, vision_feature_layer=-2,
                     vision_feature_select_strategy="default", projector_hidden_act="gelu")
    lc._attn_implementation = "sdpa"
    m = LlavaForConditionalGeneration(lc)
    m.load_state_dict(build_to_hf_llama(P, m.state_dict(), t, vc.used_layers))
    batch = O.make_batch(cfg, 2, 45, seed=1)
    with torch.no_grad():
        hf32 = m(**batch).loss.item()
        with torch.autocast("cpu", dtype=torch.bfloat16):
            hf16 = m(**batch).loss.item()
        o32 = O.forward_loss(P, cfg, batch, "fp32").item()
        o16 = O.forward_loss(P, cfg, batch, "bf16").item()
    assert abs(o32 - hf32) < 2e-6, (o32, hf32)
    assert abs(o16 - hf16) < 2e-6, (o16, hf16)
    _grads_match(P, cfg, batch, m,
                 lambda G: build_to_hf_llama(G, dict(m.state_dict()), t, vc.used_layers))


def test_gate_up_blocking_roundtrip():
    g, u = torch.randn(384, 8), torch.randn(384, 8)
    w = O.block_gate_up(g, u)
    assert torch.equal(w[:128], g[:128]) and torch.equal(w[128:256], u[:128])
    g2, u2 = O.unblock_gate_up(w, 384)
    assert torch.equal(g, g2) and torch.equal(u, u2)
