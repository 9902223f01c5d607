"""ORACLE fixture generator, round 3 — run in the build container only (test
infrastructure; nothing here ships or runs on the product path).

Adds to tests/golden/fullsize_r3.json (SURVEY.md §8(c)(iii) full-size scalar goldens):

  * `noise` for the round-2 training scalars (c3train, c2train of fullsize_r2.json): the
    bf16 rounding-noise sigma of EVERY quantity (step-1 grad norm, the two step losses,
    the loss after them) — the std of the oracle's bf16-autocast run over n weight
    perturbations w·(1 + 1e-7·N(0,1)) (the fp32 values do not move).  The GPU tests hold
    each quantity to |HIP − HF bf16| < 1e-4 + 2σ_q (absolute).
  * `c5train`: BASELINE C5 = CLIP-ViT-L/14-336 + Pythia-2.8B @ 576 + 511 tokens, M = 2,
    AdamW (the LLaVA-pretrain recipe's optimizer, src/models/llava.py:96-104, effective
    wd 0), lr 1e-4 for two steps, no clip: step-1 grad norm, step losses, loss after —
    bf16 and fp32, with σ per quantity.  (The GPU test runs it with sharding zero_3 +
    offload at world 1, the reference's C5 DeepSpeed setting, src/train.py:182-213.)
  * `llava-pretrain` / `llava-pretrain-M16`: the reference's own model (src/models/
    llava.py:22-58: CLIP-ViT-L/14-336 + Llama-3.2-1B, built from explicit
    hyper-parameters), forward loss fp32 / bf16 of the real HF LlavaForConditionalGeneration
    and of the oracle, with σ; `llava-pretrain-train`: tower and LLM frozen (llava.py:49-52),
    AdamW lr 1e-3 (the recipe's) for two steps on the projector: projector grad norm, step
    losses, loss after, bf16 / fp32, σ per quantity.

Memory (62 GB container, no swap): the C5 runs keep the fp32 Adam moments in memory-mapped
files under $GOLDEN_SCRATCH (default /tmp/mmpt_golden), regenerate the weights per run
instead of holding a second copy, and drop each gradient once its parameter is updated.
The optimizer is `adam_step_`, a restatement of torch's single-tensor Adam/AdamW
(torch/optim/adam.py _single_tensor_adam, foreach=False) that tests/test_oracle_golden.py
checks bitwise against torch.optim.AdamW / Adam.

Usage: GOLDEN_ONLY=noise|c5train|llava python oracle/gen_golden_r3.py
"""

from __future__ import annotations

import json
import os
import statistics
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

from oracle import model as O  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
REL = 1e-7  # weight perturbation of the noise runs (relative)


def adam_step_(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, step: int,
               lr: float, betas: tuple[float, float], eps: float, weight_decay: float,
               decoupled: bool) -> None:
    """torch.optim.Adam(W) single-tensor update, in place (torch/optim/adam.py
    _single_tensor_adam, capturable=False, amsgrad=False, maximize=False): `step` is the
    step count AFTER the increment."""
    b1, b2 = betas
    if weight_decay != 0:
        if decoupled:
            p.mul_(1 - lr * weight_decay)
        else:
            g = g.add(p, alpha=weight_decay)
    m.lerp_(g, 1 - b1)
    v.mul_(b2).addcmul_(g, g, value=1 - b2)
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    step_size = lr / bc1
    denom = (v.sqrt() / (bc2 ** 0.5)).add_(eps)
    p.addcdiv_(m, denom, value=-step_size)


class _State:
    """Adam moments per parameter: in RAM, or memory-mapped files (zero-initialised, like
    torch's lazily created state) when `scratch` is set."""

    def __init__(self, scratch: str | None):
        self.scratch = scratch
        self.mv: dict[str, tuple[torch.Tensor, torch.Tensor]] = {}
        if scratch:
            os.makedirs(scratch, exist_ok=True)

    def get(self, name: str, like: torch.Tensor):
        if name not in self.mv:
            if self.scratch:
                pair = []
                for k in "mv":
                    path = os.path.join(self.scratch, f"{name}.{k}")
                    arr = np.memmap(path, dtype=np.float32, mode="w+", shape=tuple(like.shape))
                    pair.append(torch.from_numpy(arr))  # zero-filled by the file system
                self.mv[name] = (pair[0], pair[1])
            else:
                self.mv[name] = (torch.zeros_like(like), torch.zeros_like(like))
        return self.mv[name]

    def close(self):
        self.mv.clear()
        if self.scratch:
            for f in os.listdir(self.scratch):
                os.remove(os.path.join(self.scratch, f))


def _perturb_(params: dict, seed: int | None) -> None:
    if seed is None:
        return
    g = torch.Generator().manual_seed(100 + seed)
    with torch.no_grad():
        for w in params.values():
            if w.is_floating_point():
                w.mul_(1 + REL * torch.randn(w.shape, generator=g))


def train_scalars(make_params, ocfg, batches, kind: str, lrs, betas, clip: float,
                  precision: str, trainable=None, perturb: int | None = None,
                  scratch: str | None = None) -> dict:
    """The reference step (src/benchmarking/utils.py:61-80) on the oracle with gradient
    accumulation over `batches`: loss = Σ CE / label tokens of the step's batch (HF
    num_items_in_batch) → backward per micro-batch → [clip] → Adam(W) → zero_grad.
    `trainable(name)` marks the parameters that train (the rest are frozen: no gradient,
    no optimizer state).  Returns the step-1 gradient L2 norm (fp64 accumulation, before
    clipping), the step losses and the loss after the steps (forward only)."""
    params = make_params()
    _perturb_(params, perturb)
    names = [n for n in params if trainable is None or trainable(n)]
    for n in names:
        params[n].requires_grad_()
    st = _State(scratch)
    n_items = sum(int((b["labels"][:, 1:] != -100).sum()) for b in batches)
    losses, gnorm = [], None
    for i, lr in enumerate(lrs):
        tot = 0.0
        for b in batches:
            loss = O.forward_loss(params, ocfg, b, precision, num_items=n_items)
            loss.backward()
            tot += loss.item()
            del loss
        if i == 0:
            gnorm = sum(float(params[n].grad.double().pow(2).sum()) for n in names) ** 0.5
        if clip > 0:
            torch.nn.utils.clip_grad_norm_([params[n] for n in names], clip)
        with torch.no_grad():
            for n in names:
                p = params[n]
                g = p.grad
                m, v = st.get(n, p)
                adam_step_(p, g, m, v, i + 1, lr, betas, 1e-8, 0.0, kind == "adamw")
                p.grad = None
        losses.append(tot)
        print(f"    {precision} step {i}: loss {tot:.7f} gnorm {gnorm}", flush=True)
    with torch.no_grad():
        after = sum(O.forward_loss(params, ocfg, b, precision, num_items=n_items).item()
                    for b in batches)
    st.close()
    del params
    return {"grad_norm": gnorm, "losses": losses, "loss_after": after}


def noise(make_params, ocfg, batches, n: int, base: dict | None = None, **kw) -> dict:
    """σ per quantity of the bf16 training scalars: the sample std over the unperturbed run
    `base` (the golden itself, one draw of the same rounding noise) and n weight
    perturbations; the per-run values are kept (`samples`)."""
    runs = [] if base is None else [base]
    for s in range(n):
        t0 = time.time()
        runs.append(train_scalars(make_params, ocfg, batches, precision="bf16", perturb=s, **kw))
        print(f"  noise run {s}: {runs[-1]} ({time.time() - t0:.0f} s)", flush=True)
    sd = statistics.stdev
    return {"grad_norm": sd([r["grad_norm"] for r in runs]),
            "losses": [sd([r["losses"][i] for r in runs]) for i in range(len(runs[0]["losses"]))],
            "loss_after": sd([r["loss_after"] for r in runs]), "n": len(runs), "rel": REL,
            "definition": "sample std over the unperturbed bf16 run and the weight "
                          "perturbations w*(1 + rel*N(0,1))",
            "samples": runs}


def forward_noise(P, ocfg, batch, n: int) -> float:
    out = []
    with torch.no_grad():
        for s in range(n):
            P2 = {k: v.clone() for k, v in P.items()}
            _perturb_(P2, s)
            out.append(O.forward_loss(P2, ocfg, batch, "bf16").item())
            del P2
    return statistics.pstdev(out)


# ---------------------------------------------------------------------------------- configs
def c3_cfg():
    return O.MMCfg(vision=O.VisionCfg(), text=O.TextCfg())


def c2_cfg():
    return O.MMCfg(vision=None, text=O.TextCfg())


def c5_cfg():
    return O.MMCfg(vision=O.VisionCfg(hidden=1024, layers=24, heads=16, ffn=4096, image=336,
                                      patch=14, eps=1e-5, act="quick_gelu", pre_ln=True,
                                      patch_bias=False),
                   text=O.TextCfg(hidden=2560, layers=32, heads=32, ffn=10240))


LLAMA_ROPE = (32.0, 1.0, 4.0, 8192)  # Llama-3.2-1B rope_scaling (llama3)


def llava_cfg():
    """llava-pretrain (src/models/llava.py:22-58): CLIP-ViT-L/14-336 tower + Llama-3.2-1B
    (h 2048, 16 layers, 32 q / 8 kv heads, F 8192, rope θ 5e5 llama3-scaled, tied
    embeddings), vocabulary 128256 + the <image> token = 128257 rows, padded to 128264."""
    t = O.TextCfg(hidden=2048, layers=16, heads=32, ffn=8192, vocab=128264, vocab_valid=128257,
                  rotary_pct=1.0, rope_theta=500000.0, eps=1e-5, arch="llama", kv_heads=8,
                  rope_scaling=LLAMA_ROPE, tie_embeddings=True)
    return O.MMCfg(vision=c5_cfg().vision, text=t, image_token_id=128256)


def _hf_llava_llama(ocfg):
    from transformers import CLIPVisionConfig, LlamaConfig, LlavaConfig, LlavaForConditionalGeneration

    t = ocfg.text
    tc = LlamaConfig(vocab_size=t.n_vocab, hidden_size=t.hidden, intermediate_size=t.ffn,
                     num_hidden_layers=t.layers, num_attention_heads=t.heads,
                     num_key_value_heads=t.n_kv, hidden_act="silu", max_position_embeddings=131072,
                     rms_norm_eps=t.eps, tie_word_embeddings=True,
                     rope_parameters={"rope_type": "llama3", "rope_theta": t.rope_theta,
                                      "factor": LLAMA_ROPE[0], "low_freq_factor": LLAMA_ROPE[1],
                                      "high_freq_factor": LLAMA_ROPE[2],
                                      "original_max_position_embeddings": LLAMA_ROPE[3]})
    vc = CLIPVisionConfig(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
                          intermediate_size=4096, image_size=336, patch_size=14,
                          hidden_act="quick_gelu", layer_norm_eps=1e-5)
    lc = LlavaConfig(vision_config=vc, text_config=tc, image_token_id=ocfg.image_token_id,
                     vision_feature_layer=-2, vision_feature_select_strategy="default",
                     projector_hidden_act="gelu")
    lc._attn_implementation = "sdpa"
    return LlavaForConditionalGeneration(lc)


def _split(full: dict, parts: int) -> list[dict]:
    n = full["input_ids"].shape[0] // parts
    return [{k: v[i * n:(i + 1) * n] for k, v in full.items()} for i in range(parts)]


# ---------------------------------------------------------------------------------- jobs
def main():
    torch.set_num_threads(int(os.environ.get("GOLDEN_THREADS", "6")))
    path = os.path.join(OUT, "fullsize_r3.json")
    try:
        with open(path) as f:
            results = json.load(f)
    except (OSError, ValueError):
        results = {}

    def save():
        import transformers

        results["generator"] = "oracle/gen_golden_r3.py"
        results["transformers"] = transformers.__version__
        with open(path, "w") as f:
            json.dump(results, f, indent=1)

    only = os.environ.get("GOLDEN_ONLY", "")
    nn = int(os.environ.get("GOLDEN_NOISE_N", "4"))
    scratch = os.environ.get("GOLDEN_SCRATCH", "/tmp/mmpt_golden")
    if only in ("", "noise"):
        jobs = {"c2train": (c2_cfg, 1, 2049, 1, "adam", (0.9, 0.95), 1.0),
                "c3train": (c3_cfg, 16, 511, 2, "adamw", (0.9, 0.999), 0.0)}
        with open(os.path.join(OUT, "fullsize_r2.json")) as f:
            r2 = json.load(f)
        for key, (mk, M, L, parts, kind, betas, clip) in jobs.items():
            if "samples" in results.get(f"{key}_noise", {}):
                continue
            ocfg = mk()
            batches = _split(O.make_batch(ocfg, M, L, seed=1), parts)
            if key == "c2train" and "c2train_reproduces_r2" not in results:
                # the restated optimizer reproduces the r2 torch.optim run
                r0 = train_scalars(lambda: O.init_params(ocfg, seed=0), ocfg, batches, kind, [1e-4, 1e-4],
                                   betas, clip, "bf16")
                with open(os.path.join(OUT, "fullsize_r2.json")) as f:
                    r2 = json.load(f)["c2train"]["bf16"]
                results["c2train_reproduces_r2"] = r0 == r2
                print("c2train reproduces r2:", r0 == r2, r0, r2, flush=True)
            print(f"{key} noise", flush=True)
            results[f"{key}_noise"] = noise(lambda: O.init_params(ocfg, seed=0), ocfg, batches, nn,
                                            base=r2[key]["bf16"], kind=kind, lrs=[1e-4, 1e-4],
                                            betas=betas, clip=clip)
            save()
    if only in ("", "c5train") and "c5train" in results and \
            "samples" not in results["c5train"]["noise"]:
        ocfg = c5_cfg()
        batches = [O.make_batch(ocfg, 2, 511, seed=1)]
        kw = dict(kind="adamw", lrs=[1e-4, 1e-4], betas=(0.9, 0.999), clip=0.0, scratch=scratch)
        print("c5train noise (with samples)", flush=True)
        results["c5train"]["noise"] = noise(lambda: O.init_params(ocfg, seed=0), ocfg, batches,
                                            int(os.environ.get("GOLDEN_NOISE_N5", "6")),
                                            base=results["c5train"]["bf16"], **kw)
        save()
    if only in ("", "c5train") and "c5train" not in results:
        ocfg = c5_cfg()
        batches = [O.make_batch(ocfg, 2, 511, seed=1)]
        rec = {"batch": "oracle.make_batch(seed=1, M=2, text_len=511)",
               "weights": "oracle.init_params(seed=0)", "optimizer": "AdamW",
               "betas": [0.9, 0.999], "lrs": [1e-4, 1e-4], "clip": 0.0}
        kw = dict(kind="adamw", lrs=[1e-4, 1e-4], betas=(0.9, 0.999), clip=0.0, scratch=scratch)
        mk = lambda: O.init_params(ocfg, seed=0)  # noqa: E731
        for prec in ("bf16", "fp32"):
            print(f"c5train {prec}", flush=True)
            rec[prec] = train_scalars(mk, ocfg, batches, precision=prec, **kw)
            results["c5train"] = rec
            save()
        rec["noise"] = noise(mk, ocfg, batches, max(3, nn - 1), base=rec["bf16"], **kw)
        results["c5train"] = rec
        save()
    if only in ("", "llava"):
        from oracle.hf_mapping import build_to_hf_llama

        ocfg = llava_cfg()
        P = O.init_params(ocfg, seed=0)
        if "llava-pretrain" not in results:
            m = _hf_llava_llama(ocfg)
            m.load_state_dict(build_to_hf_llama(P, m.state_dict(), ocfg.text, ocfg.vision.used_layers))
            for key, M in (("llava-pretrain", 2), ("llava-pretrain-M16", 16)):
                bt = O.make_batch(ocfg, M, 511, seed=1)
                with torch.no_grad():
                    rec = {"batch": f"oracle.make_batch(seed=1, M={M}, text_len=511)",
                           "weights": "oracle.init_params(seed=0)",
                           "loss_fp32": m(**bt).loss.item()}
                    with torch.autocast("cpu", dtype=torch.bfloat16):
                        rec["loss_bf16_autocast"] = m(**bt).loss.item()
                    rec["oracle_loss_fp32"] = O.forward_loss(P, ocfg, bt, "fp32").item()
                    rec["oracle_loss_bf16_autocast"] = O.forward_loss(P, ocfg, bt, "bf16").item()
                print(key, rec, flush=True)
                results[key] = rec
                save()
            del m
            for key, M in (("llava-pretrain", 2), ("llava-pretrain-M16", 16)):
                bt = O.make_batch(ocfg, M, 511, seed=1)
                results[key]["bf16_noise_std"] = forward_noise(P, ocfg, bt, nn)
                print(key, results[key], flush=True)
                save()
        if "llava-pretrain-train" in results and \
                "samples" not in results["llava-pretrain-train"]["noise"]:
            batches = _split(O.make_batch(ocfg, 16, 511, seed=1), 2)
            kw = dict(kind="adamw", lrs=[1e-3, 1e-3], betas=(0.9, 0.999), clip=0.0,
                      trainable=lambda n: n.startswith("proj."))
            rec = results["llava-pretrain-train"]
            rec["noise"] = noise(lambda: {k: v.clone() for k, v in P.items()}, ocfg, batches, nn,
                                 base=rec["bf16"], **kw)
            save()
        if "llava-pretrain-train" not in results:
            batches = _split(O.make_batch(ocfg, 16, 511, seed=1), 2)
            rec = {"batch": "oracle.make_batch(seed=1, M=16, text_len=511) as 2 x 8",
                   "weights": "oracle.init_params(seed=0)", "optimizer": "AdamW",
                   "betas": [0.9, 0.999], "lrs": [1e-3, 1e-3], "clip": 0.0,
                   "trainable": "proj.* (tower and LLM frozen, src/models/llava.py:49-52)"}
            kw = dict(kind="adamw", lrs=[1e-3, 1e-3], betas=(0.9, 0.999), clip=0.0,
                      trainable=lambda n: n.startswith("proj."))
            mk = lambda: {k: v.clone() for k, v in P.items()}  # noqa: E731
            for prec in ("bf16", "fp32"):
                print(f"llava-pretrain-train {prec}", flush=True)
                rec[prec] = train_scalars(mk, ocfg, batches, precision=prec, **kw)
            rec["noise"] = noise(mk, ocfg, batches, nn, base=rec["bf16"], **kw)
            results["llava-pretrain-train"] = rec
            save()
    save()


if __name__ == "__main__":
    main()
