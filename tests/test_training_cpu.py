"""BASELINE C1: `pythia-160m --methods naive`, world size 1, on the CPU through
scripts/training.py (the reference's scripts/training.py:73-104: model class →
TrainingArguments JSON → Trainer.train()), dummy dataset, micro-batch 1.

The CLI runs two optimizer steps from the TrainingArguments JSON that
scripts/to_training_arguments.py writes for the naive method; the losses are checked
against the same two steps of transformers' GPTNeoXForCausalLM driven directly
(torch.optim.Adam with the Pythia kwargs and weight decay 0 as HF's parameter groups
apply it, the cosine_with_min_lr schedule, clip 1.0) on the same dummy samples."""

import json
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_c1_pythia160m_naive_cpu(tmp_path):
    args = tmp_path / "args.json"
    subprocess.run([sys.executable, "scripts/to_training_arguments.py", "--output", str(args),
                    "--micro-batch-size", "1", "--gradient-accumulation-steps", "1",
                    "--num-nodes", "1", "--gpus-per-node", "1", "--gpu-type", "mi355x",
                    "--model", "pythia-160m"], cwd=ROOT, check=True, timeout=120)
    targs = json.load(open(args))
    assert targs["per_device_train_batch_size"] == 1 and not targs.get("torch_compile")
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="8")
    out = subprocess.run([sys.executable, "scripts/training.py", "--output-dir", str(tmp_path / "o"),
                          "--model-type", "pythia-160m", "--training-arguments", str(args),
                          "--max-steps", "2", "--cpu"], cwd=ROOT, env=env, capture_output=True,
                         text=True, timeout=600)
    assert out.returncode == 0, out.stderr
    log = [json.loads(ln) for ln in open(tmp_path / "o" / "trainer_log.jsonl")]
    assert [r["step"] for r in log] == [1, 2] and all(r["device"] == "cpu" for r in log)

    # the same two steps, driven directly on transformers' GPTNeoXForCausalLM
    sys.path.insert(0, ROOT)
    from transformers import GPTNeoXConfig, GPTNeoXForCausalLM

    from multimodal_llm_pretraining_amd.models import get_model_class
    from multimodal_llm_pretraining_amd.optim import lr_lambda

    torch.set_num_threads(8)
    mc = get_model_class("pythia-160m")
    torch.manual_seed(int(targs.get("seed", 42)))
    m = GPTNeoXForCausalLM(GPTNeoXConfig(
        vocab_size=50304, hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
        intermediate_size=3072, rotary_pct=0.25, rotary_emb_base=10000,
        max_position_embeddings=2048, use_parallel_residual=True, hidden_act="gelu",
        layer_norm_eps=1e-5, tie_word_embeddings=False, attn_implementation="eager"))
    kw = dict(mc.optimizer_kwargs, weight_decay=0.0)
    opt = torch.optim.Adam(m.parameters(), **kw)
    ds = mc.load_dummy_dataset()
    sk = targs.get("lr_scheduler_kwargs") or {}
    ref = []
    for step in range(2):
        lr = kw["lr"] * lr_lambda(targs["lr_scheduler_type"], step, targs.get("warmup_steps", 0),
                                  targs["max_steps"], sk.get("min_lr_rate", 0.0))
        for gr in opt.param_groups:
            gr["lr"] = lr
        it = ds[step]
        b = {k: v.unsqueeze(0) for k, v in it.items()}
        loss = m(**b).loss
        loss.backward()
        torch.nn.utils.clip_grad_norm_(m.parameters(), targs["max_grad_norm"])
        opt.step()
        opt.zero_grad(set_to_none=True)
        ref.append(loss.item())
        assert abs(log[step]["learning_rate"] - lr) < 1e-12
    for got, want in zip((r["loss"] for r in log), ref):
        assert abs(got - want) < 1e-5, (got, want)
