"""Model plugin surface (§8(a) row a8, §8(b) item 1): the reference's
`BaseModelClass` / `get_model_class` API (src/models/__init__.py:67-162, 240-296)
for the model types whose training step runs on the MI355X path, plus the
drop-in model object `build_model(use_custom_kernels=True)` returns.

Recipes restate the reference's constants: Pythia (src/models/pythia.py:14-98) and
the LLaVA-pretrain recipe (src/models/llava.py:80-124) used for the C3 composition
"vit-b16-pythia-1b" (ViT-B/16 + Pythia-1B).

`use_custom_kernels=True`  → `MMPTForPretraining`: an nn.Module whose parameters are
    views of ONE flat fp32 buffer (params.ParamStore) and whose forward/backward run
    the HIP engine (engine.Engine) through a single autograd node.
`use_custom_kernels=False` → the plain transformers model built from explicit
    configs (the reference's "naive" branch: eager attention); no fetch.
`llava-pretrain` is the reference's own CLIP-L/14-336 + Llama-3.2-1B model (with its
freeze); model types outside the path (roberta, mamba, convnext, vit, llava-finetune,
vilt-*) raise.
"""

from __future__ import annotations

from abc import ABC, abstractmethod
from types import SimpleNamespace
from typing import Any, Literal

import torch
import torch.nn as nn

from . import config as C
from .data import DummyMultimodalLanguageModelingDataset, DummyTextModelingDataset
from .engine import Batch, Engine
from .params import ParamStore, init_normal

PythiaT = Literal["pythia-14m", "pythia-31m", "pythia-70m", "pythia-160m", "pythia-410m",
                  "pythia-1b", "pythia-1.4b", "pythia-2.8b", "pythia-6.9b", "pythia-12b"]
VitPythiaT = Literal["vit-b16-pythia-1b", "clip-l14-336-pythia-2.8b"]
LlavaT = Literal["llava-pretrain", "llava-pretrain-unfrozen"]
ModelT = Literal[PythiaT, VitPythiaT, LlavaT]
# reference model types that are not on this path (out of scope;
# llava-finetune needs a private checkpoint, src/models/llava.py:151)
OUT_OF_SCOPE = ("roberta", "mamba", "convnext-large-1k", "convnext-large-22k",
                "convnext-xlarge-22k", "vit", "llava-finetune",
                "vilt-pretrain", "vilt-finetune", "vilt-original-pretrain",
                "vilt-original-finetune")


class BaseModelClass(ABC):
    """Same properties and meaning as the reference's BaseModelClass."""

    def __init__(self, model_type: str) -> None:
        self.model_type = model_type

    @abstractmethod
    def build_model(self, use_custom_kernels: bool = True) -> nn.Module: ...

    @property
    def supports_activation_checkpointing(self) -> bool:
        return True

    @property
    def supports_compilation(self) -> bool:
        return True

    @property
    @abstractmethod
    def batch_size(self) -> int: ...

    @property
    @abstractmethod
    def training_steps(self) -> int: ...

    @property
    @abstractmethod
    def mixed_precision(self) -> Literal[None, "bf16", "fp16"]: ...

    @property
    @abstractmethod
    def optimizer(self) -> type[torch.optim.Optimizer]: ...

    @property
    @abstractmethod
    def optimizer_kwargs(self) -> dict[str, Any]: ...

    @property
    @abstractmethod
    def scheduler_type(self) -> str: ...

    @property
    @abstractmethod
    def scheduler_kwargs(self) -> dict[str, Any]: ...

    @property
    @abstractmethod
    def max_grad_norm(self) -> float: ...

    @property
    def hf_training_args(self) -> dict[str, Any]:
        return {}

    @property
    @abstractmethod
    def fsdp_layers_to_wrap(self) -> list[str]: ...

    @abstractmethod
    def load_dummy_dataset(self): ...

    # build-side extension: the engine configuration behind build_model()
    @property
    def model_config(self) -> C.ModelConfig:
        return C.get_config(self.model_type)


class PythiaModelClass(BaseModelClass):
    """src/models/pythia.py:14-98 (GPTNeoX, Adam, cosine_with_min_lr, clip 1.0)."""

    _LR = {"pythia-14m": 1.0e-3, "pythia-31m": 1.0e-3, "pythia-70m": 1.0e-3,
           "pythia-160m": 6.0e-4, "pythia-410m": 3.0e-4, "pythia-1b": 3.0e-4,
           "pythia-1.4b": 2.0e-4, "pythia-2.8b": 1.6e-4, "pythia-6.9b": 1.2e-4,
           "pythia-12b": 1.2e-4}

    def build_model(self, use_custom_kernels: bool = True) -> nn.Module:
        if use_custom_kernels:
            return MMPTForPretraining(self.model_config)
        return build_hf_model(self.model_config)

    batch_size = property(lambda self: 1024)
    training_steps = property(lambda self: 143000)

    @property
    def mixed_precision(self):
        # Pythia README: fp16 for every size except pythia-1b (bf16)
        return "bf16" if self.model_type == "pythia-1b" else "fp16"

    optimizer = property(lambda self: torch.optim.Adam)

    @property
    def optimizer_kwargs(self):
        return {"lr": self._LR[self.model_type], "betas": (0.9, 0.95), "eps": 1e-8,
                "weight_decay": 0.01}

    scheduler_type = property(lambda self: "cosine_with_min_lr")

    @property
    def scheduler_kwargs(self):
        return {"num_warmup_steps": int(0.01 * self.training_steps), "min_lr_rate": 0.1}

    max_grad_norm = property(lambda self: 1.0)
    fsdp_layers_to_wrap = property(lambda self: ["GPTNeoXLayer"])
    vocab_size = property(lambda self: 50304)
    sequence_length = property(lambda self: 2049)

    def load_dummy_dataset(self, num_samples: int = 50_000):
        return DummyTextModelingDataset(self.vocab_size, self.sequence_length, num_samples)


class VitPythiaModelClass(BaseModelClass):
    """C3: ViT-B/16 + Pythia-1B joined by the LLaVA projector, trained with the
    LLaVA-pretrain recipe of src/models/llava.py:80-124 (batch 256, 2180 steps, bf16,
    AdamW lr 1e-3 wd 0, cosine with 3% warmup, no clipping)."""

    def build_model(self, use_custom_kernels: bool = True) -> nn.Module:
        if use_custom_kernels:
            return MMPTForPretraining(self.model_config)
        return build_hf_model(self.model_config)

    batch_size = property(lambda self: 256)
    training_steps = property(lambda self: 2180)
    mixed_precision = property(lambda self: "bf16")
    optimizer = property(lambda self: torch.optim.AdamW)
    optimizer_kwargs = property(lambda self: {"lr": 1e-3, "weight_decay": 0.0})
    scheduler_type = property(lambda self: "cosine")

    @property
    def scheduler_kwargs(self):
        return {"num_warmup_steps": int(self.training_steps * 0.03)}

    max_grad_norm = property(lambda self: 0.0)
    fsdp_layers_to_wrap = property(lambda self: ["GPTNeoXLayer", "ViTLayer"])
    vocab_size = property(lambda self: 50304)
    image_size = property(lambda self: self.model_config.vision.image)
    image_token_index = property(lambda self: 50303)

    @property
    def sequence_length(self) -> int:  # 196 image slots + 511 text tokens
        return self.model_config.vision.num_patches + 511

    def load_dummy_dataset(self, num_samples: int = 20_000):
        v = self.model_config.vision
        return DummyMultimodalLanguageModelingDataset(
            vocab_size=self.vocab_size, sequence_length=self.sequence_length,
            image_size=self.image_size, num_samples=num_samples,
            image_token_id=self.image_token_index, image_tokens=v.num_patches)


class ClipPythiaModelClass(VitPythiaModelClass):
    """C5: CLIP-ViT-L/14-336 (the reference llava-pretrain tower, src/models/llava.py:24-45)
    + Pythia-2.8B, LLaVA-pretrain recipe (576 image slots + 511 text tokens)."""

    fsdp_layers_to_wrap = property(lambda self: ["GPTNeoXLayer", "CLIPEncoderLayer"])


class LlavaPretrainModelClass(VitPythiaModelClass):
    """The reference's own image-text model, `llava-pretrain` (src/models/llava.py:22-146):
    CLIP-ViT-L/14-336 tower + 2-layer GELU projector + Llama-3.2-1B, built from explicit
    hyper-parameters (no hub fetch), with the reference's added "<image>" token
    (vocabulary 128256 + 1, image token 128256; padded to 128264 rows) and its recipe: batch
    256, 2180 steps, bf16, AdamW lr 1e-3 wd 0, cosine with 3% warmup, no clipping.

    Freeze: under the reference's pinned transformers 4.47.1, `build_model` freezes every
    parameter whose name starts with "vision_tower" or "language_model"
    (src/models/llava.py:49-52), so only the projector trains — `llava-pretrain` reproduces
    that (ModelConfig.freeze_tower_and_llm).  `llava-pretrain-unfrozen` trains everything,
    which is what the same code does under transformers 5.x, whose parameter names no longer
    carry those prefixes."""

    fsdp_layers_to_wrap = property(lambda self: ["LlamaDecoderLayer"])
    vocab_size = property(lambda self: 128257)  # 128256 + "<image>"
    image_token_index = property(lambda self: 128256)


def get_model_class(model_type: str) -> BaseModelClass:
    """src/models/__init__.py:240-296 for the types on the MI355X path."""
    if model_type in PythiaModelClass._LR:
        return PythiaModelClass(model_type)
    if model_type == "vit-b16-pythia-1b":
        return VitPythiaModelClass(model_type)
    if model_type == "clip-l14-336-pythia-2.8b":
        return ClipPythiaModelClass(model_type)
    if model_type in ("llava-pretrain", "llava-pretrain-unfrozen"):
        return LlavaPretrainModelClass(model_type)
    if model_type in OUT_OF_SCOPE:
        raise NotImplementedError(f"model type {model_type!r} is not on the MI355X hot path "
                                  "(SURVEY.md §8 scope)")
    raise ValueError(f"unknown model type {model_type!r}")


# ------------------------------------------------------------------ drop-in model object
class _EngineStep(torch.autograd.Function):
    """One autograd node for the whole model: forward = Engine.forward (loss and the
    fused CE gradient), backward = Engine.backward (accumulates into the flat grads)."""

    @staticmethod
    def forward(ctx, model, batch, denom, *params):
        loss_sum = model.engine.forward(batch, 1.0 / denom, need_grad=True)
        ctx.model, ctx.batch = model, batch
        return (loss_sum / denom).view(())

    @staticmethod
    def backward(ctx, gout):
        m = ctx.model
        m._attach_grads()
        m.engine.backward(ctx.batch, scale=gout)
        ctx.model = ctx.batch = None
        return (None, None, None) + (None,) * len(m._plist)


class MMPTOutput(dict):
    """ModelOutput-like: `.loss` and `.get("loss")` (src/benchmarking/flops.py:34)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e


class MMPTForPretraining(nn.Module):
    """Drop-in for the `PreTrainedModel` that build_model returns (§8(b) 'what the
    model object must provide'): forward(input_ids, pixel_values, attention_mask,
    labels, num_items_in_batch) → output with .loss; `.config.hidden_size` /
    `.config.text_config.hidden_size`; gradient_checkpointing_enable();
    parameters named like the flat store (state_dict keys = ParamStore names).

    Gradients live in the store's flat fp32 buffer; every `p.grad` is a view of it.
    `zero_grad(set_to_none=True)` (the torch default) is honoured: the next backward
    zeroes the buffer and re-attaches the views."""

    supports_gradient_checkpointing = True
    _no_split_modules = ["GPTNeoXLayer", "ViTLayer"]

    def __init__(self, cfg: C.ModelConfig, device: torch.device | str = "cuda", seed: int = 0,
                 world: int | None = None):
        super().__init__()
        import torch.distributed as dist

        if world is None:
            world = dist.get_world_size() if dist.is_initialized() else 1
        self.mmpt_config = cfg
        self.store = ParamStore(C.param_shapes(cfg), device, world=world,
                                trainable=cfg.trainable if cfg.freeze_tower_and_llm else None)
        init_normal(self.store, seed, cfg=cfg)
        self.engine = Engine(cfg, self.store)
        self._plist: list[nn.Parameter] = []
        for name in self.store.names():
            parent = self
            *path, leaf = name.split(".")
            for part in path:
                if not hasattr(parent, part):
                    parent.add_module(part, nn.Module())
                parent = getattr(parent, part)
            prm = nn.Parameter(self.store.p(name),  # aliases the flat master buffer
                               requires_grad=cfg.trainable(name))
            prm._mmpt_store = self.store
            parent.register_parameter(leaf, prm)
            self._plist.append(prm)
        self._grad_views = [self.store.g(n) for n in self.store.names()]
        self._attach_grads()
        t = cfg.text
        text_cfg = SimpleNamespace(hidden_size=t.hidden, num_hidden_layers=t.layers,
                                   num_attention_heads=t.heads, intermediate_size=t.ffn,
                                   vocab_size=t.n_vocab, rotary_pct=t.rotary_pct,
                                   num_key_value_heads=t.n_kv, model_type=t.arch)
        self.config = SimpleNamespace(hidden_size=t.hidden, text_config=text_cfg,
                                      use_cache=False, model_type="mmpt",
                                      image_token_index=cfg.image_token_id)
        self.gradient_checkpointing = False
        self._shadow_version = self.store.master._version

    # -- HF-compatible knobs
    def gradient_checkpointing_enable(self, gradient_checkpointing_kwargs=None):
        """Per-layer activation checkpointing: each ViT / GPTNeoX layer keeps only its
        input and recomputes its forward right before its backward (Engine.checkpointing)."""
        self.gradient_checkpointing = True
        self.engine.checkpointing = True

    def gradient_checkpointing_disable(self):
        self.gradient_checkpointing = False
        self.engine.checkpointing = False

    # -- ZeRO-3 hand-over
    def partition_out(self) -> dict[str, torch.Tensor]:
        """Hand the weights to a ZeRO-3 trainer and release this object's full-size device
        storage (fp32 master, bf16 shadows, fp32 grads ≈ 12 B/param), the way DeepSpeed
        ZeRO-3 replaces each parameter's data by an empty placeholder once it is
        partitioned.  Returns the fp32 weights as a CPU state dict (the Zero3Store loads
        its slice of it); afterwards the step runs through the trainer only."""
        sd = {n: self.store.p(n).detach().to("cpu", copy=True) for n in self.store.names()}
        dev = self.store.device
        for p in self._plist:
            p.grad = None
            p.data = torch.empty(0, dtype=torch.float32, device=dev)
        self._grad_views = []
        for attr in ("master", "grad", "shadow", "shadow_t"):
            setattr(self.store, attr, torch.empty(0, device=dev))
        self.partitioned = True
        if dev.type == "cuda":
            torch.cuda.empty_cache()
        return sd

    partitioned = False

    # -- gradients
    def _attach_grads(self):
        live = [p for p in self._plist if p.requires_grad]
        if live and live[0].grad is None:
            self.store.zero_grad()
        for p, g in zip(self._plist, self._grad_views):
            if not p.requires_grad:  # frozen (llava-pretrain): no .grad, like HF
                continue
            if p.grad is None or p.grad.data_ptr() != g.data_ptr():
                p.grad = g

    # -- parameters changed outside the fused optimizer (e.g. torch.optim.Adam in place)
    def _refresh_if_stale(self):
        v = self.store.master._version
        if v != self._shadow_version:
            self.store.refresh_shadow()
            self._shadow_version = v

    def forward(self, input_ids=None, labels=None, pixel_values=None, attention_mask=None,
                num_items_in_batch=None, **unused):
        if self.partitioned:
            raise RuntimeError("parameters were partitioned out to a ZeRO-3 trainer "
                               "(partition_out): run the step through that trainer")
        if labels is None:
            raise ValueError("the pre-training step needs labels (loss is the output)")
        if attention_mask is not None and not bool((attention_mask != 0).all()):
            raise NotImplementedError("padded attention masks are not on the path "
                                      "(dummy/pre-training batches are unpadded)")
        self._refresh_if_stale()
        batch = Batch(self.mmpt_config, input_ids, labels, pixel_values, self.store.device)
        denom = float(num_items_in_batch) if num_items_in_batch is not None \
            else float(max(1, batch.num_items))
        if torch.is_grad_enabled() and any(p.requires_grad for p in self._plist):
            loss = _EngineStep.apply(self, batch, denom, *self._plist)
        else:  # evaluation: no dlogits, no activation cache
            loss = (self.engine.forward(batch, 1.0 / denom, need_grad=False) / denom).view(())
        return MMPTOutput(loss=loss)


def build_hf_model(cfg: C.ModelConfig) -> nn.Module:
    """The reference's use_custom_kernels=False branch: plain transformers modules from
    explicit configs (eager attention), no hub access."""
    from transformers import GPTNeoXConfig, GPTNeoXForCausalLM

    t = cfg.text
    tc = GPTNeoXConfig(vocab_size=t.vocab, hidden_size=t.hidden, num_hidden_layers=t.layers,
                       num_attention_heads=t.heads, intermediate_size=t.ffn,
                       rotary_pct=t.rotary_pct, rotary_emb_base=t.rope_theta,
                       max_position_embeddings=2048, use_parallel_residual=True,
                       hidden_act="gelu", layer_norm_eps=t.eps, tie_word_embeddings=False,
                       attn_implementation="eager")
    if cfg.vision is None:
        return GPTNeoXForCausalLM(tc)
    from transformers import LlavaConfig, LlavaForConditionalGeneration, ViTConfig

    v = cfg.vision
    vc = ViTConfig(hidden_size=v.hidden, num_hidden_layers=v.layers, num_attention_heads=v.heads,
                   intermediate_size=v.ffn, image_size=v.image, patch_size=v.patch,
                   attn_implementation="eager")
    lc = LlavaConfig(vision_config=vc, text_config=tc, image_token_id=cfg.image_token_id,
                     vision_feature_layer=v.feature_layer,
                     vision_feature_select_strategy="default", projector_hidden_act="gelu")
    return LlavaForConditionalGeneration(lc)
