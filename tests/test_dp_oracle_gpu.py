"""Every data-parallel mode against the CPU oracle (src/train.py:126-213):
two ranks share cuda:0 over a gloo group (RCCL refuses two ranks on one device — the
exchange issues the same torch.distributed calls the RCCL run makes; tests/test_rccl_gpu.py
drives the same code over RCCL at world 1 with every collective forced), each rank takes
half of a 4-sample batch, gradient clipping at 1.0, two optimizer steps.

Checked against oracle.train_steps (one process, the whole 4-sample batch, HF bf16
autocast; src/benchmarking/utils.py:61-80): the two step losses and the loss of a third
batch after the two updates.  Tolerance: 2 × the bf16 floor |oracle bf16 - oracle fp32|
(the HIP step and the CPU bf16 autocast are two independent bf16 roundings of the same fp32
computation, each about that far from fp32, so they can sit on opposite sides of it —
measured: step-1 loss HIP 7.00714, CPU bf16 7.00745, fp32 7.00725) plus 1e-4 (step 1) /
3e-4 (later: Adam's first steps move every weight by ≈lr, so bf16 rounding differences in
the gradients show up in the next loss).

Modes: ddp (layer-wise all-reduce overlapped with the backward), zero_1 (reduce-scatter
after the backward), zero_2 (ZeRO-3's per-unit gradient reduce-scatter, replicated bf16
weights re-gathered per unit after each step), zero_3
(per-unit gather / reduce-scatter), zero_2 + optimizer offload (host Adam), and the Llama
side (tied embedding: the lm_head and the input embedding share one gradient) under ddp
and zero_2.
"""

import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

from oracle import model as O

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_parity_gpu import oracle_cfg  # noqa: E402

pytestmark = pytest.mark.gpu

CLIP, LR, STEPS = 1.0, 1e-3, 2
TEXT_LEN = {"tiny-mm": 40, "tiny-llama": 96}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(name):
    from multimodal_llm_pretraining_amd import config as C

    ocfg = oracle_cfg(C.get_config(name))
    batches = [O.make_batch(ocfg, 4, TEXT_LEN[name], seed=s) for s in range(1, STEPS + 2)]
    return ocfg, O.init_params(ocfg, seed=0), batches


def _sl(bd, sl):
    return {k: v[sl] for k, v in bd.items()}


def _worker(rank, world, port, name, sharding, offload, q):
    import torch.distributed as dist

    from multimodal_llm_pretraining_amd.optim import AdamConfig
    from multimodal_llm_pretraining_amd.trainer import ManualTrainer, StepConfig

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _, P, batches = _setup(name)
        tr = ManualTrainer(StepConfig(model=name, sharding=sharding, scheduler="constant",
                                      offload=offload),
                           AdamConfig(lr=LR, max_grad_norm=CLIP), "cuda", init=False)
        tr.store.load(P)
        tr.store.refresh_shadow()
        tr.store.refresh_transposed()
        losses = []
        for bd in batches[:STEPS]:
            full = tr.stage(bd)
            mine = tr.stage(_sl(bd, slice(2 * rank, 2 * rank + 2)))
            s = tr.train_step([mine], full.num_items).cpu()
            dist.all_reduce(s)  # per-rank CE sums → global
            losses.append(s.item() / full.num_items)
        ev = tr.stage(batches[STEPS])
        after = tr.engine.forward(ev, 1.0 / ev.num_items, need_grad=False).item() / ev.num_items
        torch.cuda.synchronize()
        q.put((rank, losses, after, dict(getattr(tr.sync, "stats", {})), None))
    except Exception:
        import traceback

        q.put((rank, None, None, None, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


_ORACLE: dict = {}


def _oracle(name):
    if name not in _ORACLE:
        ocfg, P, batches = _setup(name)
        opt = O.OptimCfg(kind="adamw", lr=LR, max_grad_norm=CLIP)
        out = {}
        for prec in ("bf16", "fp32"):
            losses, Pn = O.train_steps(P, ocfg, batches[:STEPS], opt, [LR] * STEPS, prec)
            with torch.no_grad():
                after = O.forward_loss(Pn, ocfg, batches[STEPS], prec).item()
            out[prec] = losses + [after]
        _ORACLE[name] = out
    return _ORACLE[name]


@pytest.mark.parametrize("name,sharding,offload", [
    ("tiny-mm", "", False), ("tiny-mm", "zero_1", False), ("tiny-mm", "zero_2", False),
    ("tiny-mm", "zero_3", False), ("tiny-mm", "zero_2", True), ("tiny-mm", "zero_3", True),
    ("tiny-llama", "", False), ("tiny-llama", "zero_2", False)])
def test_two_ranks_match_oracle(name, sharding, offload):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, sharding, offload, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, losses, after, overlapped, err = q.get(timeout=300)
        assert err is None, err
        res[r] = (losses + [after], overlapped)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _oracle(name)
    for r, (got, overlapped) in res.items():
        print(f"rank {r} {sharding or 'ddp'}{'+offload' if offload else ''}: HIP {got} "
              f"oracle bf16 {ref['bf16']} fp32 {ref['fp32']}")
        for i, (g, b, f) in enumerate(zip(got, ref["bf16"], ref["fp32"])):
            tol = (1e-4 if i == 0 else 3e-4) + 2 * abs(b - f)
            assert abs(g - b) < tol, (r, i, g, b, f)
        if sharding == "zero_2":
            # ZeRO-2: every unit reduce-scattered once per micro-batch, and all-gathered
            # once per step before its first use (steps 2.. and the evaluation forward)
            assert overlapped["reduce_scatters"] == overlapped["gathers"] > 0, overlapped
