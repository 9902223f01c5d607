"""DeepSpeed memory semantics that decide the sweep's max-micro-batch and feasibility
results (VERDICT r02 missing #3; src/train.py:172-181 stage 2 `reduce_scatter` /
`contiguous_gradients`, :203-207 `offload_optimizer`):

* optimizer offload keeps no fp32 master on the device past the region the step reads as
  fp32 (LayerNorm / embeddings): 12 B/param leave the device (master, m, v), not 8;
* ZeRO-2 partitions the fp32 master AND the gradients (no rank holds a full fp32 gradient
  or master buffer), unlike ZeRO-1, which reduce-scatters a full gradient buffer.

Each configuration runs in its own process (its own caching-allocator statistics); the
allocator's measured difference between two configurations must equal the difference of
the device buffers their stores / optimizers hold, so the memory is really gone.
"""

import math
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

NAME = "tiny-mm"


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _device_bytes(*objs) -> int:
    """bytes of the distinct CUDA tensors (or lists of them) held as attributes of objs"""
    seen, total = set(), 0
    for o in objs:
        for v in vars(o).values():
            for t in (v if isinstance(v, (list, tuple)) else [v]):
                if isinstance(t, torch.Tensor) and t.is_cuda and t.numel():
                    key = t.untyped_storage().data_ptr()
                    if key not in seen:
                        seen.add(key)
                        total += t.untyped_storage().nbytes()
    return total


def _worker(rank, world, port, sharding, offload, keep_master, q):
    import torch.distributed as dist

    from multimodal_llm_pretraining_amd import config as C
    from multimodal_llm_pretraining_amd.optim import AdamConfig
    from multimodal_llm_pretraining_amd.trainer import ManualTrainer, StepConfig
    from oracle import model as O
    from test_parity_gpu import oracle_cfg

    os.environ["MMPT_OFFLOAD_KEEP_MASTER"] = "1" if keep_master else "0"
    os.environ["MMPT_OFFLOAD_ASYNC"] = "0"  # no host thread racing the measurements
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        tr = ManualTrainer(StepConfig(model=NAME, sharding=sharding, scheduler="constant",
                                      offload=offload), AdamConfig(lr=1e-3), "cuda:0")
        ocfg = oracle_cfg(C.get_config(NAME))
        b = tr.stage(O.make_batch(ocfg, 2, 40, seed=1))
        for _ in range(2):
            tr.train_step([b], b.num_items * world)
        tr.flush()
        torch.cuda.synchronize()
        st = tr.store
        q.put((rank, {"alloc": torch.cuda.memory_allocated(),
                      "held": _device_bytes(st, tr.opt, tr.sync),
                      "padded": getattr(st, "padded", None), "numel": st.numel,
                      "fp32_end": st.fp32_end, "fp32_keep": getattr(st, "fp32_keep", st.fp32_end),
                      "fp32_units": list(getattr(st, "fp32_units", [])),
                      "params": sum(math.prod(s) for s in st.shapes.values()),
                      "master": st.master.numel(), "grad": st.grad.numel()}, None))
    except Exception:
        import traceback

        q.put((rank, None, traceback.format_exc()))
    finally:
        if world > 1:
            dist.destroy_process_group()


def _run(sharding, offload, keep_master, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, sharding, offload, keep_master, q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, rec, err = q.get(timeout=300)
        assert err is None, err
        out[r] = rec
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


@pytest.mark.parametrize("sharding", ["", "zero_3"])
def test_offload_releases_device_master(sharding):
    kept = _run(sharding, True, True, 1)[0]
    rel = _run(sharding, True, False, 1)[0]
    # only what the step reads as fp32 stays on the device: the persistent region (+ under
    # ZeRO-3 this rank's shards of the fp32 units, DeepSpeed's partitioned embeddings)
    assert rel["master"] == rel["fp32_keep"] and kept["master"] > rel["master"]
    freed = (kept["master"] - rel["master"]) * 4
    assert kept["held"] - rel["held"] == freed
    # the caching allocator sees exactly those bytes gone
    assert abs((kept["alloc"] - rel["alloc"]) - freed) <= 1 << 20, (kept, rel, freed)


def test_zero2_partitions_master_and_grads_two_ranks():
    z1 = _run("zero_1", False, True, 2)
    z2 = _run("zero_2", False, True, 2)
    for r in range(2):
        a, b = z1[r], z2[r]
        # ZeRO-1: full fp32 master and gradient buffers on every rank
        assert a["master"] == a["grad"] == a["padded"]
        # ZeRO-2: the replicated fp32-read region + this rank's half of every unit
        assert b["master"] == b["grad"] == b["numel"] < a["padded"] // 2 + b["fp32_end"] + 4096
        # the allocator's difference is the difference of the buffers the stores hold (at
        # this tiny size ZeRO-2's two per-unit gradient windows cost about what the halved
        # master and gradients save; the full-size balance is test_zero2_memory_model_cpu's)
        assert abs((a["alloc"] - b["alloc"]) - (a["held"] - b["held"])) <= 4 << 20, (a, b)


@pytest.mark.parametrize("sharding", ["zero_2", "zero_3"])
def test_embeddings_partitioned_above_persistence_threshold(sharding):
    """DeepSpeed's stage3_param_persistence_threshold (10 x hidden, src/train.py:182-194):
    an fp32-read parameter above 10 x the text hidden size (the token embedding; the ViT
    position embedding at full size) is not replicated under ZeRO-2/3 — each rank holds half
    of its fp32 master, gradient and Adam state at 2 ranks; only the small fp32-read
    parameters (LayerNorm, CLS, and here the tiny model's 17 x 128 position table) stay whole
    on every rank."""
    from multimodal_llm_pretraining_amd import config as C
    from multimodal_llm_pretraining_amd.params import is_fp32_read

    cfg = C.get_config(NAME)
    shapes = C.param_shapes(cfg)
    big = {n for n, sh in shapes.items() if is_fp32_read(n) and math.prod(sh) > 10 * cfg.text.hidden}
    assert "text.embed" in big
    out = _run(sharding, False, True, 2)
    for r in range(2):
        a = out[r]
        assert set(a["fp32_units"]) == big, (a, big)
        # per rank: the small replicated region + half of everything else (+ padding)
        assert a["master"] == a["grad"] == a["numel"]
        assert a["numel"] < (a["params"] - a["fp32_end"]) // 2 + a["fp32_end"] + 64 * 2 * 40, a
        assert a["fp32_end"] < 0.05 * a["params"], a
