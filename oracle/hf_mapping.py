"""ORACLE — test infrastructure only.

State-dict mapping between HF transformers 5.15 module names
(LlavaForConditionalGeneration(ViT, GPTNeoX) / GPTNeoXForCausalLM) and the
build's flat parameter layout (names differ across transformers
versions; 4.47 used `attention.attention.query` for ViT, 5.x `q_proj`).

ViT q/k/v projections are stacked into one [3h, h] "qkv" matrix (planar q|k|v);
the Conv2d patch weight is flattened to [h, C·p·p] (im2col order (c, ky, kx)).
"""

from __future__ import annotations

import torch


def hf_to_build(sd: dict[str, torch.Tensor], vision_layers_used: int | None,
                text_layers: int, multimodal: bool) -> dict[str, torch.Tensor]:
    out: dict[str, torch.Tensor] = {}
    if multimodal:
        vt = "model.vision_tower."
        lm = "model.language_model."
        head = "lm_head.weight"
        w = sd[vt + "embeddings.patch_embeddings.projection.weight"]
        out["vision.patch.weight"] = w.reshape(w.shape[0], -1).clone()
        out["vision.patch.bias"] = sd[vt + "embeddings.patch_embeddings.projection.bias"].clone()
        out["vision.cls"] = sd[vt + "embeddings.cls_token"].reshape(-1).clone()
        out["vision.pos"] = sd[vt + "embeddings.position_embeddings"][0].clone()
        for i in range(vision_layers_used or 0):
            p = f"{vt}layers.{i}."
            q = f"vision.layers.{i}."
            out[q + "ln1.weight"] = sd[p + "layernorm_before.weight"].clone()
            out[q + "ln1.bias"] = sd[p + "layernorm_before.bias"].clone()
            out[q + "qkv.weight"] = torch.cat([sd[p + f"attention.{n}_proj.weight"] for n in "qkv"], 0)
            out[q + "qkv.bias"] = torch.cat([sd[p + f"attention.{n}_proj.bias"] for n in "qkv"], 0)
            out[q + "o.weight"] = sd[p + "attention.o_proj.weight"].clone()
            out[q + "o.bias"] = sd[p + "attention.o_proj.bias"].clone()
            out[q + "ln2.weight"] = sd[p + "layernorm_after.weight"].clone()
            out[q + "ln2.bias"] = sd[p + "layernorm_after.bias"].clone()
            out[q + "fc1.weight"] = sd[p + "mlp.fc1.weight"].clone()
            out[q + "fc1.bias"] = sd[p + "mlp.fc1.bias"].clone()
            out[q + "fc2.weight"] = sd[p + "mlp.fc2.weight"].clone()
            out[q + "fc2.bias"] = sd[p + "mlp.fc2.bias"].clone()
        pj = "model.multi_modal_projector."
        out["proj.fc1.weight"] = sd[pj + "linear_1.weight"].clone()
        out["proj.fc1.bias"] = sd[pj + "linear_1.bias"].clone()
        out["proj.fc2.weight"] = sd[pj + "linear_2.weight"].clone()
        out["proj.fc2.bias"] = sd[pj + "linear_2.bias"].clone()
    else:
        lm = "gpt_neox."
        head = "embed_out.weight" if "embed_out.weight" in sd else "lm_head.weight"
    out["text.embed"] = sd[lm + "embed_in.weight"].clone()
    for i in range(text_layers):
        p = f"{lm}layers.{i}."
        q = f"text.layers.{i}."
        out[q + "ln1.weight"] = sd[p + "input_layernorm.weight"].clone()
        out[q + "ln1.bias"] = sd[p + "input_layernorm.bias"].clone()
        out[q + "ln2.weight"] = sd[p + "post_attention_layernorm.weight"].clone()
        out[q + "ln2.bias"] = sd[p + "post_attention_layernorm.bias"].clone()
        out[q + "qkv.weight"] = sd[p + "attention.query_key_value.weight"].clone()
        out[q + "qkv.bias"] = sd[p + "attention.query_key_value.bias"].clone()
        out[q + "dense.weight"] = sd[p + "attention.dense.weight"].clone()
        out[q + "dense.bias"] = sd[p + "attention.dense.bias"].clone()
        out[q + "fc1.weight"] = sd[p + "mlp.dense_h_to_4h.weight"].clone()
        out[q + "fc1.bias"] = sd[p + "mlp.dense_h_to_4h.bias"].clone()
        out[q + "fc2.weight"] = sd[p + "mlp.dense_4h_to_h.weight"].clone()
        out[q + "fc2.bias"] = sd[p + "mlp.dense_4h_to_h.bias"].clone()
    out["text.final_ln.weight"] = sd[lm + "final_layer_norm.weight"].clone()
    out["text.final_ln.bias"] = sd[lm + "final_layer_norm.bias"].clone()
    out["text.lm_head"] = sd[head].clone()
    return out


def build_to_hf(P: dict[str, torch.Tensor], hf_sd: dict[str, torch.Tensor], vision_layers_used: int | None,
                text_layers: int, multimodal: bool) -> dict[str, torch.Tensor]:
    """Inverse of hf_to_build: returns a full HF state dict whose mapped entries are
    taken from the build layout `P` (unused HF modules keep their `hf_sd` values)."""
    out = {k: v.clone() for k, v in hf_sd.items()}
    lm = "model.language_model." if multimodal else "gpt_neox."
    if multimodal and "model.vision_tower.embeddings.class_embedding" in hf_sd:
        _clip_to_hf(P, out, vision_layers_used or 0)
        multimodal_vit = False
    else:
        multimodal_vit = multimodal
    if multimodal:
        pj = "model.multi_modal_projector."
        out[pj + "linear_1.weight"] = P["proj.fc1.weight"].clone()
        out[pj + "linear_1.bias"] = P["proj.fc1.bias"].clone()
        out[pj + "linear_2.weight"] = P["proj.fc2.weight"].clone()
        out[pj + "linear_2.bias"] = P["proj.fc2.bias"].clone()
    if multimodal_vit:
        vt = "model.vision_tower."
        w = out[vt + "embeddings.patch_embeddings.projection.weight"]
        out[vt + "embeddings.patch_embeddings.projection.weight"] = P["vision.patch.weight"].view_as(w).clone()
        out[vt + "embeddings.patch_embeddings.projection.bias"] = P["vision.patch.bias"].clone()
        out[vt + "embeddings.cls_token"] = P["vision.cls"].view(1, 1, -1).clone()
        out[vt + "embeddings.position_embeddings"] = P["vision.pos"].unsqueeze(0).clone()
        for i in range(vision_layers_used or 0):
            p, q = f"{vt}layers.{i}.", f"vision.layers.{i}."
            out[p + "layernorm_before.weight"] = P[q + "ln1.weight"].clone()
            out[p + "layernorm_before.bias"] = P[q + "ln1.bias"].clone()
            h = P[q + "o.weight"].shape[0]
            for j, n in enumerate("qkv"):
                out[p + f"attention.{n}_proj.weight"] = P[q + "qkv.weight"][j * h:(j + 1) * h].clone()
                out[p + f"attention.{n}_proj.bias"] = P[q + "qkv.bias"][j * h:(j + 1) * h].clone()
            out[p + "attention.o_proj.weight"] = P[q + "o.weight"].clone()
            out[p + "attention.o_proj.bias"] = P[q + "o.bias"].clone()
            out[p + "layernorm_after.weight"] = P[q + "ln2.weight"].clone()
            out[p + "layernorm_after.bias"] = P[q + "ln2.bias"].clone()
            out[p + "mlp.fc1.weight"] = P[q + "fc1.weight"].clone()
            out[p + "mlp.fc1.bias"] = P[q + "fc1.bias"].clone()
            out[p + "mlp.fc2.weight"] = P[q + "fc2.weight"].clone()
            out[p + "mlp.fc2.bias"] = P[q + "fc2.bias"].clone()
    head = "lm_head.weight" if multimodal else (
        "embed_out.weight" if "embed_out.weight" in hf_sd else "lm_head.weight")
    out[lm + "embed_in.weight"] = P["text.embed"].clone()
    for i in range(text_layers):
        p, q = f"{lm}layers.{i}.", f"text.layers.{i}."
        out[p + "input_layernorm.weight"] = P[q + "ln1.weight"].clone()
        out[p + "input_layernorm.bias"] = P[q + "ln1.bias"].clone()
        out[p + "post_attention_layernorm.weight"] = P[q + "ln2.weight"].clone()
        out[p + "post_attention_layernorm.bias"] = P[q + "ln2.bias"].clone()
        out[p + "attention.query_key_value.weight"] = P[q + "qkv.weight"].clone()
        out[p + "attention.query_key_value.bias"] = P[q + "qkv.bias"].clone()
        out[p + "attention.dense.weight"] = P[q + "dense.weight"].clone()
        out[p + "attention.dense.bias"] = P[q + "dense.bias"].clone()
        out[p + "mlp.dense_h_to_4h.weight"] = P[q + "fc1.weight"].clone()
        out[p + "mlp.dense_h_to_4h.bias"] = P[q + "fc1.bias"].clone()
        out[p + "mlp.dense_4h_to_h.weight"] = P[q + "fc2.weight"].clone()
        out[p + "mlp.dense_4h_to_h.bias"] = P[q + "fc2.bias"].clone()
    out[lm + "final_layer_norm.weight"] = P["text.final_ln.weight"].clone()
    out[lm + "final_layer_norm.bias"] = P["text.final_ln.bias"].clone()
    out[head] = P["text.lm_head"].clone()
    return out


def _clip_to_hf(P: dict[str, torch.Tensor], out: dict[str, torch.Tensor], used: int) -> None:
    """CLIP vision tower (transformers 5.15 names under LlavaForConditionalGeneration:
    model.vision_tower.{embeddings, pre_layrnorm, encoder.layers.i.{self_attn, layer_norm1/2,
    mlp}}); the patch weight drops the build's im2col pad columns."""
    vt = "model.vision_tower."
    w = out[vt + "embeddings.patch_embedding.weight"]
    k = w[0].numel()
    out[vt + "embeddings.patch_embedding.weight"] = P["vision.patch.weight"][:, :k].reshape(w.shape).clone()
    out[vt + "embeddings.class_embedding"] = P["vision.cls"].clone()
    out[vt + "embeddings.position_embedding.weight"] = P["vision.pos"].clone()
    out[vt + "pre_layrnorm.weight"] = P["vision.ln_pre.weight"].clone()
    out[vt + "pre_layrnorm.bias"] = P["vision.ln_pre.bias"].clone()
    for i in range(used):
        p, q = f"{vt}encoder.layers.{i}.", f"vision.layers.{i}."
        out[p + "layer_norm1.weight"] = P[q + "ln1.weight"].clone()
        out[p + "layer_norm1.bias"] = P[q + "ln1.bias"].clone()
        h = P[q + "o.weight"].shape[0]
        for j, n in enumerate("qkv"):
            out[p + f"self_attn.{n}_proj.weight"] = P[q + "qkv.weight"][j * h:(j + 1) * h].clone()
            out[p + f"self_attn.{n}_proj.bias"] = P[q + "qkv.bias"][j * h:(j + 1) * h].clone()
        out[p + "self_attn.out_proj.weight"] = P[q + "o.weight"].clone()
        out[p + "self_attn.out_proj.bias"] = P[q + "o.bias"].clone()
        out[p + "layer_norm2.weight"] = P[q + "ln2.weight"].clone()
        out[p + "layer_norm2.bias"] = P[q + "ln2.bias"].clone()
        out[p + "mlp.fc1.weight"] = P[q + "fc1.weight"].clone()
        out[p + "mlp.fc1.bias"] = P[q + "fc1.bias"].clone()
        out[p + "mlp.fc2.weight"] = P[q + "fc2.weight"].clone()
        out[p + "mlp.fc2.bias"] = P[q + "fc2.bias"].clone()


def llama_to_hf(P: dict[str, torch.Tensor], out: dict[str, torch.Tensor], layers: int, ffn: int,
                heads: int, kv_heads: int, lm: str) -> None:
    """Llama text model (transformers 5.15 names: {lm}embed_tokens / layers.i.{input_layernorm,
    self_attn.{q,k,v,o}_proj, post_attention_layernorm, mlp.{gate,up,down}_proj} / norm, and
    the tied lm_head) from the build layout: the fused q|k|v rows are split, the blocked
    gate|up rows unblocked, the padded vocabulary rows dropped."""
    from oracle.model import unblock_gate_up

    V = out[lm + "embed_tokens.weight"].shape[0]
    out[lm + "embed_tokens.weight"] = P["text.embed"][:V].clone()
    for i in range(layers):
        p, q = f"{lm}layers.{i}.", f"text.layers.{i}."
        out[p + "input_layernorm.weight"] = P[q + "ln1.weight"].clone()
        out[p + "post_attention_layernorm.weight"] = P[q + "ln2.weight"].clone()
        w = P[q + "qkv.weight"]
        D = w.shape[1] // heads
        wq, wk, wv = w.split([heads * D, kv_heads * D, kv_heads * D], 0)
        out[p + "self_attn.q_proj.weight"] = wq.clone()
        out[p + "self_attn.k_proj.weight"] = wk.clone()
        out[p + "self_attn.v_proj.weight"] = wv.clone()
        out[p + "self_attn.o_proj.weight"] = P[q + "dense.weight"].clone()
        g, u = unblock_gate_up(P[q + "gate_up.weight"], ffn)
        out[p + "mlp.gate_proj.weight"] = g.clone()
        out[p + "mlp.up_proj.weight"] = u.clone()
        out[p + "mlp.down_proj.weight"] = P[q + "down.weight"].clone()
    out[lm + "norm.weight"] = P["text.final_ln.weight"].clone()
    head = P.get("text.lm_head", P["text.embed"])
    out["lm_head.weight"] = head[:V].clone()


def build_to_hf_llama(P: dict[str, torch.Tensor], hf_sd: dict[str, torch.Tensor], text, vision_used: int | None):
    """LlamaForCausalLM (vision_used None) or LlavaForConditionalGeneration(CLIP, Llama)."""
    out = {k: v.clone() for k, v in hf_sd.items()}
    if vision_used is None:
        llama_to_hf(P, out, text.layers, text.ffn, text.heads, text.n_kv, "model.")
        return out
    _clip_to_hf(P, out, vision_used)
    pj = "model.multi_modal_projector."
    out[pj + "linear_1.weight"] = P["proj.fc1.weight"].clone()
    out[pj + "linear_1.bias"] = P["proj.fc1.bias"].clone()
    out[pj + "linear_2.weight"] = P["proj.fc2.weight"].clone()
    out[pj + "linear_2.bias"] = P["proj.fc2.bias"].clone()
    llama_to_hf(P, out, text.layers, text.ffn, text.heads, text.n_kv, "model.language_model.")
    return out
