"""Model configurations of the hot path (product-owned; no HF import).

Hyper-parameters restate the public HF configs the reference loads by name
(GPTNeoXConfig.from_pretrained("EleutherAI/pythia-*"), src/models/pythia.py:18-21;
ViTConfig, src/models/vit.py:11-16) — they cannot be fetched offline, so they
are written out here (SURVEY.md §8c "Unavailable offline").
"""

from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class VisionConfig:
    """ViT encoder (tf:models/vit): pre-LN, qkv bias, erf-GELU, LN eps 1e-12."""

    hidden: int = 768
    layers: int = 12
    heads: int = 12
    ffn: int = 3072
    image: int = 224
    patch: int = 16
    channels: int = 3
    eps: float = 1e-12
    feature_layer: int = -2  # LlavaConfig.vision_feature_layer default
    # CLIP vision tower (tf:models/clip/modeling_clip.py; the reference's llava-pretrain
    # tower openai/clip-vit-large-patch14-336, src/models/llava.py:24-45): quick-GELU MLP,
    # pre_layrnorm on the embeddings, bias-free patch conv, LN eps 1e-5
    act: str = "gelu"  # "gelu" (erf) | "quick_gelu"
    pre_ln: bool = False
    patch_bias: bool = True

    @property
    def patch_k(self) -> int:
        """im2col width C·p·p padded to a multiple of 8 (16-B GEMM rows; zero columns)."""
        return (self.channels * self.patch * self.patch + 7) // 8 * 8

    @property
    def num_patches(self) -> int:
        return (self.image // self.patch) ** 2

    @property
    def head_dim(self) -> int:
        return self.hidden // self.heads

    @property
    def used_layers(self) -> int:
        """hidden_states[feature_layer] needs only the first L+1+feature_layer layers (P12)."""
        return self.layers + 1 + self.feature_layer


@dataclass(frozen=True)
class TextConfig:
    """arch "gptneox": GPTNeoX / Pythia (tf:models/gpt_neox) — parallel residual, LayerNorm,
    partial RoPE, fused per-head q|k|v with biases, erf-GELU MLP, untied lm_head.
    arch "llama": Llama-3 (tf:models/llama, the LLM of the reference's llava-pretrain,
    src/models/llava.py:25) — sequential residual, RMSNorm, GQA (kv_heads), full RoPE with
    the llama3 frequency scaling, SwiGLU MLP, no biases, lm_head tied to the embedding."""

    hidden: int = 2048
    layers: int = 16
    heads: int = 8
    ffn: int = 8192
    vocab: int = 50304
    rotary_pct: float = 0.25
    rope_theta: float = 10000.0
    eps: float = 1e-5
    arch: str = "gptneox"
    kv_heads: int = 0  # 0 = heads (no GQA)
    # llama3 rope scaling: (factor, low_freq_factor, high_freq_factor, original_max_position)
    rope_scaling: tuple | None = None
    tie_embeddings: bool = False
    vocab_valid: int = 0  # real vocabulary when `vocab` is padded to a multiple of 8 (0 = vocab)

    @property
    def head_dim(self) -> int:
        return self.hidden // self.heads

    @property
    def rot_dims(self) -> int:
        return int(self.head_dim * self.rotary_pct)

    @property
    def llama(self) -> bool:
        return self.arch == "llama"

    @property
    def n_kv(self) -> int:
        return self.kv_heads or self.heads

    @property
    def qkv_dim(self) -> int:
        return (self.heads + 2 * self.n_kv) * self.head_dim

    @property
    def n_vocab(self) -> int:
        return self.vocab_valid or self.vocab


@dataclass(frozen=True)
class ModelConfig:
    text: TextConfig
    vision: VisionConfig | None = None
    image_token_id: int = 50303  # last id of the 50304 Pythia vocab
    # LLaVA-pretrain freeze (src/models/llava.py:49-52, under the pinned transformers 4.47.1
    # names): the vision tower and the whole language model (embeddings, layers, final norm,
    # lm_head) are frozen — only the projector is trained.
    freeze_tower_and_llm: bool = False

    @property
    def multimodal(self) -> bool:
        return self.vision is not None

    def trainable(self, name: str) -> bool:
        return not self.freeze_tower_and_llm or name.startswith("proj.")


def _pythia(h, L, H, F):
    return TextConfig(hidden=h, layers=L, heads=H, ffn=F)


PYTHIA = {
    "pythia-14m": _pythia(128, 6, 4, 512),
    "pythia-31m": _pythia(256, 6, 8, 1024),
    "pythia-70m": _pythia(512, 6, 8, 2048),
    "pythia-160m": _pythia(768, 12, 12, 3072),
    "pythia-410m": _pythia(1024, 24, 16, 4096),
    "pythia-1b": _pythia(2048, 16, 8, 8192),
    "pythia-1.4b": _pythia(2048, 24, 16, 8192),
    "pythia-2.8b": _pythia(2560, 32, 32, 10240),
    "pythia-6.9b": _pythia(4096, 32, 32, 16384),
    "pythia-12b": _pythia(5120, 36, 40, 20480),
}

def _llama(h, L, H, kv, F, V, V_valid, theta=500000.0, scaling=(32.0, 1.0, 4.0, 8192),
           tie=True, eps=1e-5):
    return TextConfig(hidden=h, layers=L, heads=H, kv_heads=kv, ffn=F, vocab=V, vocab_valid=V_valid,
                      rotary_pct=1.0, rope_theta=theta, eps=eps, arch="llama", rope_scaling=scaling,
                      tie_embeddings=tie)


# meta-llama/Llama-3.2-1B(-Instruct) public config (hidden 2048, 16 layers, 32 q / 8 kv heads
# of 64, SwiGLU 8192, rope_theta 5e5 with llama3 scaling factor 32 / 1 / 4 / 8192, tied
# embeddings), with the reference's added "<image>" token (src/models/llava.py:40-45:
# 128256 + 1 = 128257 ids, image token 128256) padded to 128264 rows (16-B rows; the
# padding takes no part in the softmax)
LLAMA32_1B = _llama(2048, 16, 32, 8, 8192, 128264, 128257)

VIT_B16 = VisionConfig()
CLIP_L14_336 = VisionConfig(hidden=1024, layers=24, heads=16, ffn=4096, image=336, patch=14,
                            eps=1e-5, act="quick_gelu", pre_ln=True, patch_bias=False)

PRESETS: dict[str, ModelConfig] = {name: ModelConfig(text=t) for name, t in PYTHIA.items()}
PRESETS["vit-b16-pythia-1b"] = ModelConfig(text=PYTHIA["pythia-1b"], vision=VIT_B16)
# BASELINE C5: CLIP-ViT-L/14-336 + Pythia-2.8B (576 image tokens + text)
PRESETS["clip-l14-336-pythia-2.8b"] = ModelConfig(text=PYTHIA["pythia-2.8b"], vision=CLIP_L14_336)
# the reference's own image-text model: llava-pretrain = CLIP-ViT-L/14-336 + Llama-3.2-1B
# (src/models/llava.py:22-58), freeze semantics of the pinned transformers 4.47.1
PRESETS["llava-pretrain"] = ModelConfig(text=LLAMA32_1B, vision=CLIP_L14_336, image_token_id=128256,
                                        freeze_tower_and_llm=True)
# the same composition with every parameter trained (transformers 5.x, where the freeze's
# name prefixes no longer match: SURVEY P12)
PRESETS["llava-pretrain-unfrozen"] = ModelConfig(text=LLAMA32_1B, vision=CLIP_L14_336,
                                                 image_token_id=128256)
PRESETS["llama-3.2-1b"] = ModelConfig(text=LLAMA32_1B)
# kernel-compatible tiny configs for parity tests (head_dim 64, 80-128 step 16, 256;
# dims % 8 == 0)
PRESETS["tiny-mm"] = ModelConfig(
    text=TextConfig(hidden=512, layers=2, heads=2, ffn=1024, vocab=1024),
    vision=VisionConfig(hidden=128, layers=3, heads=2, ffn=256, image=64, patch=16),
    image_token_id=1023)
PRESETS["tiny-lm"] = ModelConfig(text=TextConfig(hidden=256, layers=2, heads=2, ffn=512, vocab=512))
# Pythia-2.8B's head shape (head_dim 80 -> padded D = 128 attention, 20 rotary dims)
PRESETS["tiny-lm-d80"] = ModelConfig(text=TextConfig(hidden=320, layers=2, heads=4, ffn=640,
                                                     vocab=512))
# C5's shapes scaled down: CLIP tower (quick-GELU, pre-LN, 14-px patches) + head_dim 80
PRESETS["tiny-clip-d80"] = ModelConfig(
    text=TextConfig(hidden=320, layers=2, heads=4, ffn=640, vocab=1024),
    vision=VisionConfig(hidden=128, layers=3, heads=2, ffn=256, image=56, patch=14, eps=1e-5,
                        act="quick_gelu", pre_ln=True, patch_bias=False),
    image_token_id=1023)


# Llama-shaped tiny configs (GQA at head_dim 64, SwiGLU F % 128 == 0, padded vocab)
PRESETS["tiny-llama"] = ModelConfig(text=_llama(256, 2, 4, 1, 256, 520, 515,
                                                scaling=(32.0, 1.0, 4.0, 64)))
PRESETS["tiny-llava"] = ModelConfig(
    text=_llama(256, 2, 4, 2, 256, 1032, 1025, scaling=(32.0, 1.0, 4.0, 64)),
    vision=VisionConfig(hidden=128, layers=3, heads=2, ffn=256, image=56, patch=14, eps=1e-5,
                        act="quick_gelu", pre_ln=True, patch_bias=False),
    image_token_id=1024)
PRESETS["tiny-llava-frozen"] = ModelConfig(text=PRESETS["tiny-llava"].text,
                                           vision=PRESETS["tiny-llava"].vision,
                                           image_token_id=1024, freeze_tower_and_llm=True)


def get_config(name: str) -> ModelConfig:
    try:
        return PRESETS[name]
    except KeyError as e:
        raise ValueError(f"unknown model {name!r}; known: {sorted(PRESETS)}") from e


def param_shapes(cfg: ModelConfig) -> dict[str, tuple[int, ...]]:
    """The build's flat state-dict layout (HF mapping: oracle/hf_mapping.py)."""
    s: dict[str, tuple[int, ...]] = {}
    t = cfg.text
    if cfg.vision is not None:
        v = cfg.vision
        s["vision.patch.weight"] = (v.hidden, v.patch_k)
        if v.patch_bias:
            s["vision.patch.bias"] = (v.hidden,)
        s["vision.cls"] = (v.hidden,)
        s["vision.pos"] = (v.num_patches + 1, v.hidden)
        if v.pre_ln:
            s["vision.ln_pre.weight"] = (v.hidden,)
            s["vision.ln_pre.bias"] = (v.hidden,)
        for i in range(v.used_layers):
            p = f"vision.layers.{i}."
            s[p + "ln1.weight"] = (v.hidden,)
            s[p + "ln1.bias"] = (v.hidden,)
            s[p + "qkv.weight"] = (3 * v.hidden, v.hidden)
            s[p + "qkv.bias"] = (3 * v.hidden,)
            s[p + "o.weight"] = (v.hidden, v.hidden)
            s[p + "o.bias"] = (v.hidden,)
            s[p + "ln2.weight"] = (v.hidden,)
            s[p + "ln2.bias"] = (v.hidden,)
            s[p + "fc1.weight"] = (v.ffn, v.hidden)
            s[p + "fc1.bias"] = (v.ffn,)
            s[p + "fc2.weight"] = (v.hidden, v.ffn)
            s[p + "fc2.bias"] = (v.hidden,)
        s["proj.fc1.weight"] = (t.hidden, v.hidden)
        s["proj.fc1.bias"] = (t.hidden,)
        s["proj.fc2.weight"] = (t.hidden, t.hidden)
        s["proj.fc2.bias"] = (t.hidden,)
    s["text.embed"] = (t.vocab, t.hidden)
    if t.llama:
        for i in range(t.layers):
            p = f"text.layers.{i}."
            s[p + "ln1.weight"] = (t.hidden,)             # input_layernorm (RMS)
            s[p + "qkv.weight"] = (t.qkv_dim, t.hidden)   # q_proj | k_proj | v_proj
            s[p + "dense.weight"] = (t.hidden, t.hidden)  # o_proj
            s[p + "ln2.weight"] = (t.hidden,)             # post_attention_layernorm (RMS)
            s[p + "gate_up.weight"] = (2 * t.ffn, t.hidden)  # gate|up, 128-row blocks
            s[p + "down.weight"] = (t.hidden, t.ffn)
        s["text.final_ln.weight"] = (t.hidden,)
        if not t.tie_embeddings:
            s["text.lm_head"] = (t.vocab, t.hidden)
        return s
    for i in range(t.layers):
        p = f"text.layers.{i}."
        s[p + "ln1.weight"] = (t.hidden,)
        s[p + "ln1.bias"] = (t.hidden,)
        s[p + "ln2.weight"] = (t.hidden,)
        s[p + "ln2.bias"] = (t.hidden,)
        s[p + "qkv.weight"] = (3 * t.hidden, t.hidden)
        s[p + "qkv.bias"] = (3 * t.hidden,)
        s[p + "dense.weight"] = (t.hidden, t.hidden)
        s[p + "dense.bias"] = (t.hidden,)
        s[p + "fc1.weight"] = (t.ffn, t.hidden)
        s[p + "fc1.bias"] = (t.ffn,)
        s[p + "fc2.weight"] = (t.hidden, t.ffn)
        s[p + "fc2.bias"] = (t.hidden,)
    s["text.final_ln.weight"] = (t.hidden,)
    s["text.final_ln.bias"] = (t.hidden,)
    s["text.lm_head"] = (t.vocab, t.hidden)
    return s


def num_params(cfg: ModelConfig) -> int:
    n = 0
    for shape in param_shapes(cfg).values():
        k = 1
        for d in shape:
            k *= d
        n += k
    return n


def flops_per_sample(cfg: ModelConfig, seq_text: int) -> float:
    """Algorithmic fwd+bwd FLOPs per sample in the reference's convention
    (src/benchmarking/flops.py:9-37: FlopCounterMode over one fwd+bwd, eager
    attention counted full-square, = 3 × forward matmul FLOPs).  ViT counts all
    `layers` because the reference instantiates (and FlopCounterMode sees) them all.
    With `freeze_tower_and_llm` (llava-pretrain, src/models/llava.py:49-52) autograd runs no
    backward in the vision tower and no weight gradients in the LLM: the count is then
    vision 1× + LLM linears 2× (forward + input gradient) + attention 3× + projector 3×."""
    t = cfg.text
    S = seq_text + (cfg.vision.num_patches if cfg.vision else 0)
    if t.llama:  # q,o: h^2 each; k,v: h*kv_dim each; gate, up, down: h*F each
        kvd = t.n_kv * t.head_dim
        lin = t.layers * 2 * S * t.hidden * (2 * t.hidden + 2 * kvd + 3 * t.ffn)
        lin += 2 * S * t.hidden * t.n_vocab
    else:
        lin = t.layers * 2 * S * t.hidden * (4 * t.hidden + 2 * t.ffn)
        lin += 2 * S * t.hidden * t.vocab
    att = t.layers * 4 * S * S * t.hidden
    vis = proj = 0.0
    if cfg.vision is not None:
        v = cfg.vision
        Sv = v.num_patches + 1
        vis = 2 * v.num_patches * v.hidden * v.channels * v.patch ** 2  # (unpadded K)
        vis += v.layers * (2 * Sv * v.hidden * (4 * v.hidden + 2 * v.ffn) + 4 * Sv * Sv * v.hidden)
        proj = 2 * v.num_patches * (v.hidden * t.hidden + t.hidden * t.hidden)
    if cfg.freeze_tower_and_llm:
        return vis + 2.0 * lin + 3.0 * att + 3.0 * proj
    return 3.0 * (lin + att + vis + proj)


def executed_flops_per_sample(cfg: ModelConfig, seq_text: int) -> float:
    """The matmul FLOPs the HIP step actually executes per sample (for `executed_mfu` beside
    the reference-convention `mfu`): lm_head + CE over the scored rows only (loss-row
    compaction: the text rows but the last for LLaVA batches), causal attention counted
    over the lower triangle with the diagonal (S(S+1)/2 score/PV pairs per head instead of
    S²), and only the vision layers the model reads (`used_layers`: vision_feature_layer
    -2 leaves the last one unbuilt).  Non-causal ViT attention stays square."""
    t = cfg.text
    n_img = cfg.vision.num_patches if cfg.vision else 0
    S = seq_text + n_img
    scored = seq_text - 1 if cfg.vision else S  # text-only batches keep every row (<5% unscored)
    head_v = t.n_vocab if t.llama else t.vocab
    if t.llama:
        kvd = t.n_kv * t.head_dim
        lin = t.layers * 2 * S * t.hidden * (2 * t.hidden + 2 * kvd + 3 * t.ffn)
    else:
        lin = t.layers * 2 * S * t.hidden * (4 * t.hidden + 2 * t.ffn)
    lin += 2 * scored * t.hidden * head_v
    att = t.layers * 4 * (S * (S + 1) / 2) * t.hidden
    vis = proj = 0.0
    if cfg.vision is not None:
        v = cfg.vision
        Sv = v.num_patches + 1
        vis = 2 * v.num_patches * v.hidden * v.channels * v.patch ** 2
        vis += v.used_layers * (2 * Sv * v.hidden * (4 * v.hidden + 2 * v.ffn) + 4 * Sv * Sv * v.hidden)
        proj = 2 * v.num_patches * (v.hidden * t.hidden + t.hidden * t.hidden)
    if cfg.freeze_tower_and_llm:
        return vis + 2.0 * lin + 3.0 * att + 3.0 * proj
    return 3.0 * (lin + att + vis + proj)
