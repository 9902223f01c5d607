#!/usr/bin/env python
"""Headline benchmark: ViT-B/16 + Pythia-1B bf16 image-text pre-training step on
1/2/4/8 MI355X (BASELINE.json `metric`, config C3).

A "step" is one optimizer step of the LLaVA-pretrain recipe (global batch 256,
src/models/llava.py:80-86): `grad_accum` micro-batches of forward+backward on every
rank (ManualTrainer.manual_training_step) + gradient exchange + fused AdamW
(manual_optimization_step), exactly the unit `estimate_step_time` extrapolates
(src/benchmarking/step_time.py:75-97) — here measured directly, synchronized.

Usage: python bench.py [--gpus N --steps K --warmup W --micro-batch M]
Multi-GPU: `python bench.py --gpus N` starts its N ranks itself (one process per GPU through
torch.distributed.run, before any GPU call — the reference's launcher does the same,
experiments/utils/distribute.py:37-61), or run it under
`python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`.
Prints ONE JSON line on rank 0.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "samples/sec/GPU + training_days, ViT-B/16+Pythia-1B bf16 at 1/2/4/8 MI355X"
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md chip table)
# workload labels of the non-headline configurations (BASELINE.json configs C2/C4/C5)
LABELS = {"vit-b16-pythia-1b": "ViT-B/16+Pythia-1B", "clip-l14-336-pythia-2.8b":
          "CLIP-ViT-L/14-336+Pythia-2.8B", "llava-pretrain": "CLIP-ViT-L/14-336+Llama-3.2-1B"}


def metric_for(model: str) -> str:
    """BASELINE.json's metric for the headline workload; the same metric, labelled with
    its own model, for the other configurations."""
    if model == "vit-b16-pythia-1b":
        return METRIC
    label = LABELS.get(model, model.replace("pythia-", "Pythia-"))
    return f"samples/sec/GPU + training_days, {label} bf16 at 1/2/4/8 MI355X"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="vit-b16-pythia-1b")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="0 = the model class's recipe batch (llava-pretrain 256, Pythia 1024)")
    ap.add_argument("--micro-batch", type=int, default=0, help="0 = largest power of two that fits (find_max_mbs_pow2), else min(64, global/N)")
    ap.add_argument("--text-len", type=int, default=0,
                    help="0 = the model class's sequence length minus the image slots")
    ap.add_argument("--sharding", default="",
                    help="'', zero_1, zero_2, zero_3, fsdp_shard_grad_op, fsdp_full_shard")
    ap.add_argument("--activation-checkpointing", action="store_true")
    ap.add_argument("--offload", action="store_true", help="optimizer state in host memory")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget-s", type=float, default=20.0)
    ap.add_argument("--no-cpu-variants", action="store_true",
                    help="skip the 1-thread and micro-batch-4 CPU baseline variants")
    ap.add_argument("--no-probe", action="store_true", help="skip per-GEMM event timing")
    ap.add_argument("--resident-inputs", action="store_true",
                    help="stage one set of micro-batches before the timed region and reuse it "
                         "every step (round-2 mode) instead of a fresh batch per step")
    ap.add_argument("--no-yardstick", action="store_true", help="skip the 8192^3 GEMM yardstick")
    return ap.parse_args()


def make_dataset(cfg, text_len: int, seed: int):
    """The reference's dummy datasets (src/benchmarking/data.py:8-21, 45-77) with the image
    placeholder pre-expanded, generated lazily per index."""
    from multimodal_llm_pretraining_amd.data import (DummyMultimodalLanguageModelingDataset,
                                                     DummyTextModelingDataset)

    if cfg.multimodal:
        v = cfg.vision
        return DummyMultimodalLanguageModelingDataset(
            vocab_size=cfg.text.n_vocab, sequence_length=text_len + v.num_patches,
            image_size=v.image, num_samples=20_000, image_token_id=cfg.image_token_id,
            image_tokens=v.num_patches, seed=seed)
    return DummyTextModelingDataset(cfg.text.n_vocab, text_len, num_samples=50_000, seed=seed)


class ClockSampler:
    """Median shader clock (MHz) over the timed region, read from the amdgpu DPM table in
    sysfs (`pp_dpm_sclk`, the active level is starred) every 50 ms by a thread; None when the
    file is not readable.  Box-to-box variance shows here first (MI355X_MICROARCH: the chip
    holds its clock below the 2.4 GHz peak under MFMA load)."""

    def __init__(self, local_rank: int):
        import glob
        import threading

        self.path = None
        try:  # the sysfs node of THIS device, by PCI address (a box may list every card)
            pr = torch.cuda.get_device_properties(local_rank)
            node = "/sys/bus/pci/devices/%04x:%02x:%02x.0/pp_dpm_sclk" % (
                pr.pci_domain_id, pr.pci_bus_id, pr.pci_device_id)
            if os.path.exists(node):
                self.path = node
        except (AttributeError, RuntimeError):
            pass
        if self.path is None:
            cards = sorted(glob.glob("/sys/class/drm/card*/device/pp_dpm_sclk"))
            if len(cards) == 1:
                self.path = cards[0]
        self.samples: list[int] = []
        self._stop = threading.Event()
        self.thread = threading.Thread(target=self._run, daemon=True) if self.path else None

    def _read(self):
        try:
            with open(self.path) as f:
                for line in f:
                    if line.rstrip().endswith("*"):
                        return int(line.split(":")[1].strip().lower().split("mhz")[0])
        except (OSError, ValueError, IndexError):
            return None
        return None

    def _run(self):
        while not self._stop.wait(0.05):
            v = self._read()
            if v is not None:
                self.samples.append(v)

    def start(self):
        if self.thread is not None:
            self.thread.start()

    def stop(self):
        if self.thread is None:
            return None
        self._stop.set()
        self.thread.join(timeout=1)
        if not self.samples:
            return None
        xs = sorted(self.samples)
        return {"median_mhz": xs[len(xs) // 2], "min_mhz": xs[0], "max_mhz": xs[-1],
                "samples": len(xs), "source": self.path}


def gemm_yardstick(device) -> dict:
    """A fixed 8192^3 bf16 GEMM of this library (gemm4p_kernel<0,0,0>) timed with HIP events
    on this box right before the timed region: the per-box reference point for comparing
    bench lines across boxes (the same code measured 260-283 samples/s on different boxes in
    round 2)."""
    from multimodal_llm_pretraining_amd import kernels as K

    n = 8192
    g = torch.Generator(device=device).manual_seed(7)
    a = torch.randn(n, n, device=device, generator=g).to(torch.bfloat16)
    b = torch.randn(n, n, device=device, generator=g).to(torch.bfloat16)
    c = torch.empty(n, n, device=device, dtype=torch.bfloat16)
    for _ in range(3):
        K.gemm(a, b, c)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record()
    for _ in range(reps):
        K.gemm(a, b, c)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    del a, b, c
    return {"shape": "8192x8192x8192 bf16 (A.B^T)", "avg_us": round(us, 1),
            "tflops": round(2 * n ** 3 / (us * 1e-6) / 1e12, 1)}


def synthetic_batch(cfg, M, text_len, device, seed):
    """DummyMultimodalLanguageModelingDataset shape (src/benchmarking/data.py:45-77), image
    tokens pre-expanded; generated directly in HBM."""
    g = torch.Generator(device=device).manual_seed(seed)
    batch = {}
    if cfg.multimodal:
        v = cfg.vision
        npch = v.num_patches
        batch["pixel_values"] = torch.rand(M, v.channels, v.image, v.image, device=device, generator=g)
        text = torch.randint(0, cfg.image_token_id, (M, text_len), device=device, generator=g)
        ids = torch.cat([torch.full((M, npch), cfg.image_token_id, device=device), text], 1)
        labels = ids.clone()
        labels[:, :npch] = -100
    else:
        ids = torch.randint(0, cfg.text.vocab, (M, text_len), device=device, generator=g)
        labels = ids.clone()
    batch["input_ids"], batch["labels"] = ids, labels
    return batch


def _oracle_cfg(cfg):
    from oracle import model as O

    v = cfg.vision
    return O.MMCfg(vision=None if v is None else O.VisionCfg(
                       hidden=v.hidden, layers=v.layers, heads=v.heads, ffn=v.ffn, image=v.image,
                       patch=v.patch, eps=v.eps, act=v.act, pre_ln=v.pre_ln,
                       patch_bias=v.patch_bias),
                   text=O.TextCfg(hidden=cfg.text.hidden, layers=cfg.text.layers,
                                  heads=cfg.text.heads, ffn=cfg.text.ffn, vocab=cfg.text.vocab,
                                  rotary_pct=cfg.text.rotary_pct),
                   image_token_id=cfg.image_token_id)


def cpu_baseline(model_name: str, text_len: int, budget_s: float, variants: bool) -> dict:
    """The oracle (torch-CPU eager restatement of the reference step, bf16 autocast, the
    model class's optimizer + clipping) timed on this host's cores on a bounded sample,
    with the reference harness semantics (step_time.py:33-72: one warm-up step, then
    timed fwd+bwd+optimizer steps):
      * main value: micro-batch 1 on all cores of the GPU box's CPU share (<= 16 threads),
        median of the steps that fit in `budget_s` (at least one, at most 5);
      * variants: micro-batch 4 on the same cores, and micro-batch 1 on ONE
        thread (the reference's .env:4 sets OMP_NUM_THREADS=1) — one timed step each."""
    from oracle import model as O
    from multimodal_llm_pretraining_amd import config as C
    from multimodal_llm_pretraining_amd.models import get_model_class

    cores = os.cpu_count() or 1
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        pass
    cores = min(cores, 16)  # the GPU box's CPU share (gpurun: 16 for one GPU)
    cfg = C.get_config(model_name)
    mc = get_model_class(model_name)
    ocfg = _oracle_cfg(cfg)
    P = O.init_params(ocfg, seed=0)
    params = [t.requires_grad_() for t in P.values()]
    kw = mc.optimizer_kwargs
    opt = mc.optimizer(params, lr=kw["lr"], betas=tuple(kw.get("betas", (0.9, 0.999))),
                       eps=kw.get("eps", 1e-8), weight_decay=0.0)  # effective wd 0
    clip = mc.max_grad_norm or 0.0
    n_img = cfg.vision.num_patches if cfg.vision else 0

    def step(batch):
        loss = O.forward_loss(P, ocfg, batch, "bf16")
        loss.backward()
        if clip > 0:
            torch.nn.utils.clip_grad_norm_(params, clip)
        opt.step()
        opt.zero_grad(set_to_none=True)

    def timed(mbs, threads, max_steps, budget):
        torch.set_num_threads(threads)
        batch = O.make_batch(ocfg, mbs, text_len, seed=1)
        times = []
        t_end = time.perf_counter() + budget
        while True:
            t0 = time.perf_counter()
            step(batch)
            times.append(time.perf_counter() - t0)
            if time.perf_counter() > t_end or len(times) >= max_steps:
                break
        times.sort()
        return times[len(times) // 2], len(times)

    torch.set_num_threads(cores)
    step(O.make_batch(ocfg, 1, text_len, seed=1))  # warm-up (allocations, first-touch)
    med, n = timed(1, cores, 5, budget_s)
    out = {"value": round(1.0 / med, 4), "unit": "samples/s", "cores": cores, "kind": "port",
           "sample": f"oracle/model.py {model_name} bf16-autocast, micro-batch 1 x "
                     f"{text_len + n_img} tokens, fwd+bwd+{mc.optimizer.__name__}, "
                     f"median of {n} step(s) after 1 warm-up",
           "sec_per_sample": round(med, 3)}
    if variants:
        out["variants"] = []
        for mbs, threads in ((4, cores), (1, 1)):
            t, n = timed(mbs, threads, 1, 0.0)
            out["variants"].append({"micro_batch": mbs, "threads": threads,
                                    "value": round(mbs / t, 4), "unit": "samples/s",
                                    "sec_per_step": round(t, 3), "steps": n})
    torch.set_num_threads(cores)
    return out


def pmc_traffic(workload: str, kernel: str):
    """L2->fabric bytes per launch (an upper bound on HBM bytes: FETCH_SIZE counts
    Infinity-Cache hits) of `kernel` from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, written by scripts/pmc_traffic.py from separate
    FETCH_SIZE / WRITE_SIZE passes of this same bench command, gfx950 FETCH_SIZE x2
    correction applied), looked up by (workload, kernel): traffic measured on another
    workload (other shapes) is never quoted.  None when not profiled."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            wl = json.load(f)["workloads"].get(workload)
        rec = wl["kernels"].get(kernel) if wl else None
    except (OSError, ValueError, KeyError):
        return None, None
    if not rec:
        return None, None
    return rec["hbm_bytes_per_launch"], f"profiles/pmc_traffic.json [{workload}] ({rec['source']})"


# Measured HBM footprint (max_memory_reserved) of the headline workload on MI355X,
# plain DP: 78 GB at micro-batch 64, 135 GB at 128, 249 GB at 256 (profiles/r01_mbs_*.json)
# -> about 21 GB fixed (params, grads, Adam state, shadows) + 0.9 GB per sample.
FOOTPRINT_GB = {"vit-b16-pythia-1b": (21.0, 0.9)}


def footprint_micro_batch(args, per_rank: int, device) -> int | None:
    """The reference's `find_max_mbs_pow2` (src/benchmarking/max_batch_size.py:11-25) from
    a measured footprint: the largest power-of-two micro-batch <= the per-rank batch that
    fits in 90% of HBM.  None for models without a measured footprint (they are probed).
    Every other mode keeps at most DDP's per-rank footprint (ZeRO shards state, offload
    moves it to the host, checkpointing keeps fewer activations), so DDP's measured model
    is an upper bound for them."""
    fp = FOOTPRINT_GB.get(args.model)
    if fp is None:
        return None
    budget_gb = 0.9 * torch.cuda.get_device_properties(device).total_memory / 1e9
    mbs = 1
    while mbs * 2 <= min(per_rank, 256) and fp[0] + fp[1] * mbs * 2 <= budget_gb:
        mbs *= 2
    return mbs


def probe_micro_batch(trainer, cfg, per_rank: int, text_len: int, device, world: int,
                      cpu_group) -> int:
    """`find_max_mbs_pow2` by probing, as the reference does (max_batch_size.py:11-25): one
    training step (fwd + bwd + optimizer) at micro-batch 1, 2, 4, ... <= the per-rank batch
    until one raises torch.cuda.OutOfMemoryError (caught; the trainer recovers its state);
    every rank must succeed (min over ranks)."""
    mbs, best = 1, 0
    while mbs <= per_rank:
        ok = 1
        try:
            b = trainer.stage(synthetic_batch(cfg, mbs, text_len, device, 7))
            trainer.train_step([b], b.num_items * world)
            trainer.flush()
            torch.cuda.synchronize(device)
            del b
        except torch.cuda.OutOfMemoryError:
            b = None
            trainer.recover()
            ok = 0
        if world > 1:
            t = torch.tensor([ok], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=cpu_group)
            ok = int(t.item())
        if not ok:
            break
        best, mbs = mbs, mbs * 2
    torch.cuda.empty_cache()
    if best == 0:
        raise SystemExit("micro-batch 1 does not fit in device memory")
    return best


def _free_port() -> int:
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def visible_gpus(environ=None, kfd_nodes: str = "/sys/class/kfd/kfd/topology/nodes",
                 render_dir: str | None = "/dev/dri") -> int | None:
    """GPUs this process may use, counted without any HIP call: the amdgpu KFD topology in
    sysfs (a node with a non-zero `gfx_target_version` is a GPU; CPU nodes have 0) whose DRM
    render node (`drm_render_minor`) this process can open — a container sees the host's whole
    topology but only its own render nodes, as the ROCm runtime does — narrowed by the
    visibility variables the HIP runtime honours (ROCR_VISIBLE_DEVICES, then
    HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES, comma-separated indices).  None when the
    topology is not readable (no amdgpu driver)."""
    import glob

    env = os.environ if environ is None else environ
    n = 0
    paths = glob.glob(os.path.join(kfd_nodes, "*", "properties"))
    if not paths:
        return None
    for path in paths:
        props = {}
        try:
            with open(path) as f:
                for line in f:
                    k, _, v = line.partition(" ")
                    props[k] = v.strip()
        except OSError:
            continue
        try:
            if int(props.get("gfx_target_version", "0")) == 0:
                continue
            minor = props.get("drm_render_minor")
            if minor is not None and int(minor) > 0 and render_dir is not None:
                node = os.path.join(render_dir, f"renderD{int(minor)}")
                if not os.access(node, os.R_OK | os.W_OK):
                    continue
        except ValueError:
            continue
        n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is not None:
            ids = [x for x in v.split(",") if x.strip() != ""]
            n = min(n, len(ids))
    return n


def self_launch(args) -> int:
    """`--gpus N > 1` without a launcher (WORLD_SIZE unset): start N ranks, one process per
    GPU, through torch.distributed.run on 127.0.0.1 (the reference launches its workers itself
    as well: experiments/utils/distribute.py:37-61, --gpus-per-node in scripts/benchmark.py:
    34-79), stream their output, and check rank 0's line reports n_gpus == N.  This process
    makes no HIP call at all: the GPUs are counted from sysfs (`visible_gpus`).
    Returns the exit code: non-zero if a rank failed or fewer than N ranks came up."""
    import subprocess

    n = args.gpus
    backend = os.environ.get("MMPT_DIST_BACKEND", "nccl")
    check = os.environ.get("MMPT_BENCH_LAUNCH_CHECK")
    if backend == "nccl" and not check:
        have = visible_gpus()
        if have is not None and have < n:
            print(f"bench.py: --gpus {n} but {have} GPU(s) visible", file=sys.stderr, flush=True)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MMPT_BENCH_SELF_LAUNCHED="1")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    line = None
    for out in proc.stdout:
        print(out, end="", flush=True)
        if out.startswith("{"):
            line = out
    rc = proc.wait()
    if rc != 0:
        return rc
    try:
        got = json.loads(line)["n_gpus"] if line else None
    except (ValueError, KeyError):
        got = None
    if got != n:
        print(f"bench.py: expected a line from {n} ranks, got n_gpus={got}", file=sys.stderr,
              flush=True)
        return 1
    return 0


def launch_check(world: int, rank: int) -> None:
    """MMPT_BENCH_LAUNCH_CHECK (CPU tests of the launcher, no GPU): every rank joins a gloo
    group and counts the ranks; rank 0 prints the line's launch fields.  =failR makes rank R
    exit with status 3 after the rendezvous (a rank that dies)."""
    mode = os.environ["MMPT_BENCH_LAUNCH_CHECK"]
    dist.init_process_group("gloo")
    t = torch.ones(1)
    dist.all_reduce(t)
    if mode == f"fail{rank}":
        sys.exit(3)
    dist.barrier()
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "ranks_seen": int(t.item()),
                          "self_launched": os.environ.get("MMPT_BENCH_SELF_LAUNCHED") == "1"}),
              flush=True)
    dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} != WORLD_SIZE {world}")
    if os.environ.get("MMPT_BENCH_LAUNCH_CHECK"):
        launch_check(world, rank)
        return
    if os.environ.get("MMPT_DIST_BACKEND", "nccl") != "nccl":
        local %= torch.cuda.device_count()  # rehearsal: ranks share the box's GPU(s)
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    # MMPT_FORCE_COLLECTIVES=1 at one GPU: a world-1 RCCL group, every exchange of the mode
    # runs (the one-GPU preview of the multi-GPU step)
    forced = os.environ.get("MMPT_FORCE_COLLECTIVES", "0") == "1"
    dist_on = world > 1 or forced
    if world == 1 and forced:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if dist_on:
        # RCCL ("nccl"); MMPT_DIST_BACKEND=gloo only to rehearse the N > 1 plumbing with
        # several ranks on one GPU (RCCL refuses two ranks on one device)
        backend = os.environ.get("MMPT_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)

    from multimodal_llm_pretraining_amd import config as C
    from multimodal_llm_pretraining_amd import kernels as K
    from multimodal_llm_pretraining_amd.optim import AdamConfig
    from multimodal_llm_pretraining_amd.trainer import ManualTrainer, StepConfig

    from multimodal_llm_pretraining_amd.models import get_model_class

    cfg = C.get_config(args.model)
    # the recipe: batch, steps, optimizer, schedule, clip (the tiny test configs — N > 1
    # rehearsals of the launch / exchange path — borrow the headline model's recipe)
    mc = get_model_class("vit-b16-pythia-1b" if args.model.startswith("tiny") else args.model)
    n_img = cfg.vision.num_patches if cfg.vision else 0
    args.global_batch = args.global_batch or mc.batch_size
    args.text_len = args.text_len or mc.sequence_length - n_img
    per_rank = args.global_batch // world
    if per_rank * world != args.global_batch:
        raise SystemExit("global batch must divide by the number of GPUs")
    mbs, mbs_rule = args.micro_batch, "--micro-batch"
    if not mbs:
        mbs, mbs_rule = footprint_micro_batch(args, per_rank, device), \
            "find_max_mbs_pow2 from the measured footprint (bench.FOOTPRINT_GB)"
    probe = not mbs
    if probe:
        mbs, mbs_rule = 1, "find_max_mbs_pow2 by OOM probing (one step per power of two)"
    if per_rank % mbs:
        raise SystemExit(f"per-rank batch {per_rank} not divisible by micro-batch {mbs}")
    ga = per_rank // mbs
    # the model class's recipe (llava-pretrain: AdamW lr 1e-3, cosine, 3% warmup, no clip,
    # src/models/llava.py:80-124; Pythia: Adam, cosine_with_min_lr, clip 1.0,
    # src/models/pythia.py:24-82), effective weight decay 0
    kw, skw = mc.optimizer_kwargs, dict(mc.scheduler_kwargs)
    trainer = ManualTrainer(
        StepConfig(model=args.model, micro_batch_size=mbs, grad_accum=ga, sharding=args.sharding,
                   activation_checkpointing=args.activation_checkpointing, offload=args.offload,
                   scheduler=mc.scheduler_type, num_warmup_steps=skw.get("num_warmup_steps", 0),
                   num_training_steps=mc.training_steps, min_lr_rate=skw.get("min_lr_rate", 0.0)),
        AdamConfig(lr=kw["lr"], betas=tuple(kw.get("betas", (0.9, 0.999))), eps=kw.get("eps", 1e-8),
                   weight_decay=0.0, adamw=mc.optimizer is torch.optim.AdamW,
                   max_grad_norm=mc.max_grad_norm or 0.0), device)
    # host-side label-token counts are summed over the ranks on a CPU (gloo) group: the
    # loss normaliser of every step is known without a device synchronisation
    cpu_group = dist.new_group(backend="gloo") if dist_on else None
    if probe:
        mbs = probe_micro_batch(trainer, cfg, per_rank, args.text_len, device, world, cpu_group)
        ga = per_rank // mbs
        trainer.step_cfg.micro_batch_size, trainer.step_cfg.grad_accum = mbs, ga

    def global_items(local: int) -> int:
        if world == 1:
            return local
        t = torch.tensor([local], dtype=torch.int64)
        dist.all_reduce(t, group=cpu_group)
        return int(t.item())

    if args.resident_inputs:
        fixed = [trainer.stage(synthetic_batch(cfg, mbs, args.text_len, device, 1000 * rank + i))
                 for i in range(ga)]
        fixed_items = global_items(sum(b.num_items for b in fixed))
        loader = copy_stream = None

        def stage_step():
            return fixed, fixed_items
    else:
        # a fresh micro-batch per micro-step from the reference's dummy dataset (a host
        # thread generates and pins it ahead, as DataLoader workers would); its staging —
        # host-to-device copies, label shift / loss-row / image maps, the device id sort of
        # the embedding backward — runs on a copy stream one step ahead, overlapped with
        # the current step, and is inside the timed region
        from multimodal_llm_pretraining_amd.data import PrefetchLoader

        loader = PrefetchLoader(make_dataset(cfg, args.text_len, seed=1), mbs, rank, world,
                                depth=ga + 1)
        copy_stream = torch.cuda.Stream(device=device)

        def stage_step():
            bs = [trainer.stage(next(loader), stream=copy_stream) for _ in range(ga)]
            return bs, global_items(sum(b.num_items for b in bs))

    nxt = stage_step()
    seq = nxt[0][0].S

    def one_step():
        nonlocal nxt
        cur, n_items = nxt
        nxt = stage_step()  # the next step's inputs, overlapped with this step
        return trainer.train_step(cur, n_items), n_items

    for _ in range(args.warmup):
        one_step()
    trainer.flush()
    torch.cuda.synchronize()
    yard = None if args.no_yardstick else gemm_yardstick(device)
    if world > 1:
        dist.barrier()
    clock = ClockSampler(local)
    from multimodal_llm_pretraining_amd.distributed import COMM_TIMER

    COMM_TIMER.on = dist_on  # per-rank comm-stream busy / exposed time (multi-GPU lines)
    if not args.no_probe:
        K.start_gemm_probe()
    clock.start()
    t0 = time.perf_counter()
    marks = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    marks[0].record()
    for i in range(args.steps):
        loss, n_items = one_step()
        marks[i + 1].record()
    trainer.flush()  # an overlapped host update of the last step belongs to the timed region
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    clock_info = clock.stop()
    comm = None
    if COMM_TIMER.on:
        COMM_TIMER.on = False
        mine = COMM_TIMER.collect()
        per_rank = [None] * world
        dist.all_gather_object(per_rank, {k: (round(v / args.steps, 3) if k.endswith("_ms") else
                                              v // args.steps) for k, v in mine.items()},
                               group=cpu_group)
        comm = {"per_step": "per rank, averaged over the timed steps",
                "busy_ms": [r["comm_busy_ms"] for r in per_rank],
                "exposed_ms": [r["comm_exposed_ms"] for r in per_rank],
                "spans": per_rank[0]["comm_spans"], "waits": per_rank[0]["comm_waits"],
                "exposed_max_ms": max(r["comm_exposed_ms"] for r in per_rank),
                "definition": "busy: HIP events on the communication stream around each "
                              "exchange; exposed: events on the compute stream around each "
                              "wait for it (the part of the exchange the step did not hide)"}
    probe = K.stop_gemm_probe()
    if loader is not None:
        loader.close()
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = t.item()

    # dominant kernel = the GEMM variant with the most device time in the timed region
    roofline = None
    if probe:
        torch.cuda.synchronize()
        agg: dict = {}
        shapes: dict = {}
        main_stream = torch.cuda.current_stream().cuda_stream
        for var, fl, by, e0, e1, shp, st in probe:
            ms = e0.elapsed_time(e1)
            side = st != main_stream  # launched beside the compute stream (weight gradients)
            if not side:  # the dominant kernel's rate comes from compute-stream launches only
                a = agg.setdefault(var, [0.0, 0.0, 0, 0.0])
                a[0] += fl
                a[1] += ms
                a[2] += 1
                a[3] += by
            sh = shapes.setdefault((var, shp, side), [0.0, 0.0, 0])
            sh[0] += fl
            sh[1] += ms
            sh[2] += 1
        var, (fl, ms, n, by) = max(agg.items(), key=lambda kv: kv[1][1])
        # per-shape table: every (kernel, M, N, K, epilogue) of the timed
        # region with its launches, average HIP-event duration and rate, by total time.
        # Launches on the weight-gradient stream overlap the compute stream's kernels: their
        # event spans include that overlap, so they carry no rate (the
        # serialised rates are the MMPT_DW_STREAM=0 trace's)
        gemm_shapes = [{"kernel": v, "M": sp[0], "N": sp[1], "K": sp[2], "epilogue": sp[3],
                        "launches_per_step": round(c / args.steps, 2),
                        "overlapped": side,
                        "avg_us": None if side else round(t * 1e3 / c, 1),
                        "tflops": None if side else round(f / (t * 1e-3) / 1e12, 1),
                        "ms_per_step": None if side else round(t / args.steps, 2)}
                       for (v, sp, side), (f, t, c) in sorted(shapes.items(), key=lambda kv: -kv[1][1])]
        serial = [(f, t) for (v, sp, side), (f, t, c) in shapes.items() if not side]
        achieved = fl / (ms * 1e-3) / 1e12
        workload = f"{args.model}|mbs{mbs}|{args.sharding or 'ddp'}"
        traffic, traffic_src = pmc_traffic(workload, var)
        roofline = {"bound": "mfma", "achieved": round(achieved, 1), "peak": PEAK_BF16_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(achieved / PEAK_BF16_TFLOPS, 4),
                    "traffic": traffic,
                    "traffic_unit": "bytes/launch, L2->fabric (rocprofv3 FETCH_SIZE x2 + "
                                    "WRITE_SIZE; includes Infinity-Cache hits, so it bounds "
                                    "HBM bytes from above)",
                    "traffic_source": traffic_src,
                    "kernel": var, "launches": n, "avg_launch_us": round(ms * 1e3 / n, 1),
                    "flops_per_launch": fl / n,
                    "algorithmic_bytes_per_launch": by / n,
                    "gemm_compute_stream_tflops": round(sum(f for f, _ in serial) /
                                                        (sum(t for _, t in serial) * 1e-3) / 1e12, 1),
                    "gemm_compute_stream_share_of_step": round(sum(t for _, t in serial) * 1e-3 / elapsed, 3),
                    "gemm_shapes": gemm_shapes}
        if any(r["overlapped"] for r in gemm_shapes):
            roofline["gemm_timing_note"] = (
                "weight-gradient GEMMs run on a second stream beside the input-gradient chain "
                "(Engine._dw): rows marked overlapped carry no rate (their event spans include "
                "the overlap); the dominant kernel and the compute-stream totals come from "
                "compute-stream launches only")
    # `frac` is the dominant kernel's (algorithmic FLOPs / its HIP-event time / peak);
    # `step_frac` is SURVEY §8(d)'s roofline.achieved: samples/s/GPU x FLOP/sample / peak

    samples = args.global_batch * args.steps
    value = samples / elapsed
    step_s = elapsed / args.steps
    fps = C.flops_per_sample(cfg, args.text_len)
    efps = C.executed_flops_per_sample(cfg, args.text_len)
    step_tflops_per_gpu = value / world * fps / 1e12
    if roofline is not None:
        roofline["scope"] = "dominant kernel: the GEMM variant with the most device time"
        roofline["step_achieved"] = round(step_tflops_per_gpu, 1)
        roofline["step_frac"] = round(step_tflops_per_gpu / PEAK_BF16_TFLOPS, 4)
    out = {
        "metric": metric_for(args.model),
        "value": round(value, 3),
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_s * 1e3, 2),
        "step_ms": [round(marks[i].elapsed_time(marks[i + 1]), 1) for i in range(args.steps)],
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (random-init weights, U[0,1) pixels, uniform token ids)",
        "inputs": ("HBM-resident: micro-batches staged once before the timed region and "
                   "reused (--resident-inputs)") if args.resident_inputs else
                  ("staged per step inside the timed region: a fresh micro-batch per micro-step "
                   "from the reference's dummy dataset (host loader thread, pinned), host-to-"
                   "device copies + label/loss-row/image maps + device id sort on a copy stream "
                   "one step ahead, overlapped with the previous step"),
        "config": {"workload": f"{args.model} " + ("LLaVA-pretrain step" if cfg.multimodal else
                                                   "causal-LM pretrain step"),
                   "global_batch": args.global_batch,
                   "micro_batch": mbs, "grad_accum": ga, "micro_batch_rule": mbs_rule,
                   "seq_len": seq,
                   "parallelism": (args.sharding or "ddp") + f"{world}" if dist_on else
                   (args.sharding or "single"),
                   **({"forced_collectives": "world-1 RCCL group, every collective of the "
                       "mode executed (MMPT_FORCE_COLLECTIVES=1)"} if forced and world == 1
                      else {}),
                   "activation_checkpointing": args.activation_checkpointing,
                   "offload": args.offload,
                   # zero_3++: int8 blockwise weight all-gather + int4 gradient all-to-all
                   **({"quantized_comm": "int8 weights / int4 grads (256-element blocks)"}
                      if args.sharding == "zero_3++" else {})},
        "samples_per_sec_per_gpu": round(value / world, 3),
        "training_days": round(mc.training_steps * step_s / 86400, 6),
        "training_steps": mc.training_steps,
        "model_tflops_per_gpu": round(step_tflops_per_gpu, 1),
        "mfu": round(step_tflops_per_gpu / PEAK_BF16_TFLOPS, 4),
        "flops_per_sample": fps,
        # the FLOPs the step executes: lm_head over the scored rows, causal attention over
        # the lower triangle, only the vision layers read (config.executed_flops_per_sample)
        "executed_flops_per_sample": efps,
        "executed_mfu": round(value / world * efps / 1e12 / PEAK_BF16_TFLOPS, 4),
        "clock": clock_info,
        "comm": comm,
        "gemm_yardstick": yard,
        "loss": round(loss.item() / n_items * world, 4) if world == 1 else None,
        "max_memory_reserved_gb": round(torch.cuda.max_memory_reserved(device) / 2**30, 1),
        "roofline": roofline,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(args.model, args.text_len, args.cpu_budget_s,
                                               not args.no_cpu_variants)
        except Exception as e:  # the baseline is reported, never the target
            out["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    if os.environ.get("MMPT_CPROFILE"):  # diagnostics: host-side profile per rank
        import cProfile
        import pstats

        prof = cProfile.Profile()
        prof.runcall(main)
        out = os.environ["MMPT_CPROFILE"] + f".rank{os.environ.get('RANK', '0')}.txt"
        with open(out, "w") as f:
            pstats.Stats(prof, stream=f).sort_stats("cumulative").print_stats(45)
    else:
        main()
