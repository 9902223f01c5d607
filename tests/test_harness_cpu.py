"""CPU tests of the reference-API harness (§8(a) rows a3-a8, a15, a16): training
arguments pinned to the reference README's JSON (tests/golden/training_arguments_readme.json,
the only fixture the reference holds for this surface), validity rules, model-class
recipes, datasets, FLOP accounting and the reference's timing formulae.

Parity note: apart from the README case, the TrainingClass / TrainingConfig outputs
are a restatement of src/train.py and experiments/config.py checked by reading;
importing the reference to generate more fixtures was denied in this environment
(DESIGN.md §Oracle), so those cases are "parity unpinned"."""

import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def _readme_args():
    with open(os.path.join(GOLDEN, "training_arguments_readme.json")) as f:
        return json.load(f)["args"]


def test_training_arguments_match_reference_readme():
    from multimodal_llm_pretraining_amd.experiments import TrainingConfig

    cfg = TrainingConfig(num_nodes=1, gpus_per_node=4, gpu_type="a100", model="pythia-1b",
                         free_lunch=True, sharding="zero_1")
    tc = cfg.training_class(micro_batch_size=16, gradient_accumulation_steps=16)
    got = json.loads(json.dumps(tc._to_huggingface_args_dict()))
    assert got == _readme_args()
    # reference quirk: num_warmup_steps is popped from scheduler_kwargs on each call
    assert tc._to_huggingface_args_dict()["warmup_steps"] == 0


def test_to_training_arguments_cli(tmp_path):
    out = tmp_path / "a" / "args.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "to_training_arguments.py"),
                    "--output", str(out), "--num-nodes", "1", "--gpus-per-node", "4",
                    "--gpu-type", "a100", "--model", "pythia-1b", "--free-lunch",
                    "--sharding", "zero_1", "--micro-batch-size", "16",
                    "--gradient-accumulation-steps", "16"], check=True, timeout=120)
    assert json.loads(out.read_text()) == _readme_args()


def test_deepspeed_and_fsdp_configs():
    from multimodal_llm_pretraining_amd.train import TrainingClass

    tc = TrainingClass(1, 1, 1, optimizer=torch.optim.AdamW, zero_stage="2")
    ds = tc._build_deepspeed_config()
    assert ds["zero_optimization"]["stage"] == 2 and ds["optimizer"]["params"]["adam_w_mode"] is True
    assert ds["zero_optimization"]["reduce_bucket_size"] == 2e8
    tc = TrainingClass(1, 1, 1, zero_stage="3", zero_offload_optimizer=True, zero_offload_params=True)
    z = tc._build_deepspeed_config()["zero_optimization"]
    assert z["stage"] == 3 and z["offload_optimizer"]["device"] == "cpu" and z["offload_param"]["pin_memory"]
    tc = TrainingClass(1, 1, 1, optimizer=torch.optim.SGD, zero_stage="1")
    assert "optimizer" not in tc._build_deepspeed_config()
    tc = TrainingClass(1, 1, 1, fsdp_sharding="full_shard", fsdp_offload=True,
                       fsdp_layers_to_wrap=["GPTNeoXLayer"])
    assert tc._build_fsdp_config() == (["full_shard", "auto_wrap", "offload"],
                                       {"transformer_layer_cls_to_wrap": ["GPTNeoXLayer"]})
    assert TrainingClass(1, 1, 1)._build_fsdp_config() == ("", None)
    assert TrainingClass(1, 1, 1)._build_deepspeed_config() is None
    with pytest.raises(TypeError):  # dict(**a, **b) with a repeated key
        TrainingClass(1, 1, 1, hf_training_args_overrides={"bf16": True})._to_huggingface_args_dict()


def test_training_class_validity():
    from multimodal_llm_pretraining_amd.train import TrainingClass

    assert TrainingClass(1, 1, 1).is_valid()
    assert not TrainingClass(0, 1, 1).is_valid()
    assert not TrainingClass(1, 1, 1, bf16=True, fp16=True).is_valid()
    assert not TrainingClass(1, 1, 1, fsdp_sharding="full_shard", zero_stage="1").is_valid()
    assert not TrainingClass(1, 1, 1, fsdp_offload=True).is_valid()
    assert not TrainingClass(1, 1, 1, zero_offload_optimizer=True).is_valid()
    assert not TrainingClass(1, 1, 1, zero_stage="2", zero_offload_params=True).is_valid()
    assert TrainingClass(1, 1, 1, zero_stage="3", zero_offload_params=True).is_valid()


def test_experiment_validity_and_sharding_map():
    from multimodal_llm_pretraining_amd.experiments import TrainingConfig, TrainingTimeEmpirical

    ok = TrainingTimeEmpirical(TrainingConfig(1, 8, "mi355x", "vit-b16-pythia-1b"))
    assert ok.is_valid() and ok.target_micro_batch_size == 32
    assert not TrainingTimeEmpirical(TrainingConfig(1, 8, "v100", "vit-b16-pythia-1b")).is_valid()
    assert not TrainingTimeEmpirical(TrainingConfig(1, 1, "mi355x", "pythia-1b", sharding="zero_1")).is_valid()
    assert not TrainingTimeEmpirical(TrainingConfig(1, 8, "mi355x", "pythia-1b", offloading=True)).is_valid()
    assert not TrainingTimeEmpirical(TrainingConfig(1, 3, "mi355x", "pythia-1b")).is_valid()
    tc = TrainingConfig(1, 8, "mi355x", "pythia-1b", free_lunch=True).training_class()
    assert tc.tf32 is False and tc.compile is True and tc.bf16
    from multimodal_llm_pretraining_amd.distributed import sharding_to_mode

    for s, mode, ex in [("", "", "ddp"), ("zero_1", "zero_1", "zero1"), ("zero_2", "zero_2", "zero2"),
                        ("zero_3", "zero_3", "zero3"), ("zero_3++", "zero_3++", "zero3"),
                        ("fsdp_shard_grad_op", "fsdp_shard_grad_op", "zero2"),
                        ("fsdp_full_shard", "fsdp_full_shard", "zero3"),
                        ("fsdp_hybrid_shard", "fsdp_hybrid_shard", "zero3"),
                        ("fsdp_hybrid_shard_zero2", "fsdp_hybrid_shard_zero2", "zero2")]:
        tc = TrainingConfig(1, 8, "mi355x", "pythia-1b", sharding=s).training_class()
        assert tc.sharding() == mode and sharding_to_mode(mode) == ex and not tc.offload()
    for s in ("zero_1", "zero_2", "zero_3", "fsdp_full_shard"):
        tc = TrainingConfig(1, 8, "mi355x", "pythia-1b", sharding=s, offloading=True).training_class()
        assert tc.offload()
    tc = TrainingConfig(1, 8, "mi355x", "pythia-1b", activation_checkpointing=True).training_class()
    assert tc.gradient_checkpointing
    with pytest.raises(NotImplementedError, match="bf16"):
        TrainingConfig(1, 8, "mi355x", "pythia-160m").training_class().build_trainer(None, None)


def test_model_classes():
    from multimodal_llm_pretraining_amd.models import get_model_class

    mc = get_model_class("vit-b16-pythia-1b")
    assert (mc.batch_size, mc.training_steps, mc.mixed_precision) == (256, 2180, "bf16")
    assert mc.optimizer is torch.optim.AdamW and mc.optimizer_kwargs == {"lr": 1e-3, "weight_decay": 0.0}
    assert mc.scheduler_type == "cosine" and mc.scheduler_kwargs == {"num_warmup_steps": 65}
    assert mc.max_grad_norm == 0.0 and mc.sequence_length == 707
    p = get_model_class("pythia-1b")
    assert p.optimizer is torch.optim.Adam and p.optimizer_kwargs["lr"] == 3e-4
    assert p.scheduler_kwargs == {"num_warmup_steps": 1430, "min_lr_rate": 0.1}
    assert get_model_class("pythia-160m").mixed_precision == "fp16"
    with pytest.raises(NotImplementedError):
        get_model_class("llava-finetune")
    # the reference's own llava-pretrain (src/models/llava.py:22-146): recipe + freeze
    lp = get_model_class("llava-pretrain")
    assert (lp.batch_size, lp.training_steps, lp.mixed_precision) == (256, 2180, "bf16")
    assert lp.optimizer is torch.optim.AdamW and lp.max_grad_norm == 0.0
    assert lp.fsdp_layers_to_wrap == ["LlamaDecoderLayer"] and lp.image_size == 336
    assert lp.model_config.freeze_tower_and_llm
    assert not get_model_class("llava-pretrain-unfrozen").model_config.freeze_tower_and_llm
    assert lp.sequence_length == 576 + 511 and lp.vocab_size == 128257
    with pytest.raises(ValueError):
        get_model_class("gpt-17")


def test_dummy_datasets():
    from multimodal_llm_pretraining_amd.models import get_model_class

    ds = get_model_class("vit-b16-pythia-1b").load_dummy_dataset(num_samples=8)
    it = ds[3]
    assert it["input_ids"].shape == (707,) and it["pixel_values"].shape == (3, 224, 224)
    assert (it["input_ids"][:196] == 50303).all() and (it["labels"][:196] == -100).all()
    assert (it["input_ids"][196:] != 50303).all() and torch.equal(it["labels"][196:], it["input_ids"][196:])
    assert float(it["pixel_values"].min()) >= 0 and float(it["pixel_values"].max()) < 1
    assert torch.equal(ds[3]["pixel_values"], it["pixel_values"])  # deterministic per index
    assert not torch.equal(ds[4]["input_ids"], it["input_ids"])
    with pytest.raises(IndexError):
        ds[8]
    t = get_model_class("pythia-1b").load_dummy_dataset(num_samples=4)[0]
    assert t["input_ids"].shape == (2049,) and torch.equal(t["labels"], t["input_ids"])
    from multimodal_llm_pretraining_amd.data import DummyMultimodalLanguageModelingDataset

    ref_layout = DummyMultimodalLanguageModelingDataset(100, 16, 32, num_samples=2, image_token_id=99)[0]
    assert ref_layout["input_ids"][0] == 99 and torch.equal(ref_layout["labels"], ref_layout["input_ids"])


def test_flops_and_training_days():
    from multimodal_llm_pretraining_amd.benchmarking import compute_training_days, count_flops_per_example
    from multimodal_llm_pretraining_amd.models import get_model_class

    # Pythia-1B@2049 = 12.818 TFLOP/sample (FlopCounterMode agrees)
    assert abs(count_flops_per_example(get_model_class("pythia-1b")) / 12.818e12 - 1) < 1e-3
    # ViT-B/16 + Pythia-1B @ 707: 4.169 TF in SURVEY (convention differences < 0.5%)
    assert abs(count_flops_per_example(get_model_class("vit-b16-pythia-1b")) / 4.169e12 - 1) < 5e-3
    assert compute_training_days(None, 10) is None
    assert compute_training_days(86.4, 1000) == pytest.approx(1.0)


def test_gpu_table():
    from multimodal_llm_pretraining_amd.gpus import ampere_or_newer_gpu, tf32_capable

    assert ampere_or_newer_gpu("mi355x") and not tf32_capable("mi355x")
    assert ampere_or_newer_gpu("a100") and tf32_capable("a100") and not ampere_or_newer_gpu("v100")
