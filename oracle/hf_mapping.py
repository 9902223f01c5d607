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
