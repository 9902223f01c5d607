"""C4's 8-rank partition on CPU (BASELINE.json configs[3]: Pythia-1B, ZeRO-3 + activation
checkpointing, 8 GPUs of one node; VERDICT r04 "next" #1): what the 8 RCCL ranks of the driver's
scaling bench will run, rehearsed with 8 gloo ranks on the tiny causal-LM config —

* the unit partition at world 8 (every unit padded to 64 x 8 elements, equal shards, the
  local layout contiguous) and DeepSpeed's persistence split (stage3_param_persistence_threshold
  "auto" = 10 x hidden, src/train.py:182-194: the token embedding above it becomes an fp32 unit,
  LayerNorm gamma/beta stay replicated);
* Zero3Sync over two accumulated micro-batches in the engine's hook order (forward: embedding,
  layers, lm_head; backward with activation checkpointing: the recompute reads the unit the
  backward acquired, so the hooks are the same): every gather window holds the exact weights,
  the gather / reduce-scatter counts follow the one-unit prefetch rule;
* the reduce-scattered gradient shards, all-gathered, equal one process accumulating the same
  16 (rank, micro-batch) contributions bit for bit (integer-valued data: fp32 sums exact in any
  order), and Σg² counts the replicated region once.

The full-size C4 layout (Pythia-1B at world 8) is checked on the meta device.  No HIP compute
is called here; the same hooks drive the HIP engine in tests/test_sharding_gpu.py.
"""

import math
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

WORLD = 8
MICRO = 2


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(world, rank):
    from multimodal_llm_pretraining_amd import config as C
    from multimodal_llm_pretraining_amd.zero3 import Zero3Store

    cfg = C.get_config("tiny-lm")
    shapes = C.param_shapes(cfg)
    st = Zero3Store(shapes, "cpu", world=world, rank=rank, persist_threshold=10 * cfg.text.hidden)
    g = torch.Generator().manual_seed(0)
    base = {n: torch.randint(-8, 9, s, generator=g).float() for n, s in shapes.items()}
    return cfg, shapes, st, base


def _order(cfg, st):
    from multimodal_llm_pretraining_amd.engine import Engine

    class _E:
        pass

    e = _E()
    e.cfg, e.s = cfg, st
    return Engine.unit_order(e)


def _run_micro_batches(st, sync, order, base, contrib):
    """The engine's hook sequence for a text-only model, MICRO micro-batches; contrib(mb) =
    the factor this process adds to every gradient.  Returns the weight mismatches seen."""
    bad = []
    f32 = set(st.fp32_units)
    for mb in range(MICRO):
        for u in order:  # forward
            sync.forward(u)
            if u in f32:
                if not torch.equal(st.p(u), base[u]):
                    bad.append(("fwd32", mb, u))
                continue
            for n in st.units[u].offsets:
                if not torch.equal(st.w(n), base[n].to(torch.bfloat16)):
                    bad.append(("fwd", mb, n))
        for u in reversed(order):  # backward (AC recompute reads the acquired unit)
            sync.backward(u)
            for n in st.units[u].offsets:
                if u not in f32 and not torch.equal(st.w(n), base[n].to(torch.bfloat16)):
                    bad.append(("bwd", mb, n))
                st.g(n).add_(base[n] * contrib(mb))
            sync.backward_done(u)
        for n in st.offsets:  # replicated (persistent) region: LayerNorms
            st.g(n).add_(base[n] * contrib(mb))
    sync.reduce_grads()
    return bad


def _worker(rank, world, port, q):
    from multimodal_llm_pretraining_amd.zero3 import Zero3Sync

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg, shapes, st, base = _setup(world, rank)
        st.load(base)
        st.shadow.copy_(st.master.to(torch.bfloat16))
        order = _order(cfg, st)
        sync = Zero3Sync(st, order)
        bad = _run_micro_batches(st, sync, order, base, lambda mb: (rank + 1) * (mb + 1))
        st.master.copy_(st.grad)
        grads = st.full_master()

        class _K:
            @staticmethod
            def sumsq_f32(x, out):
                out.copy_((x.double() ** 2).sum().float().view(1))

        ss = sync.global_sumsq(_K).item()
        q.put((rank, bad, {n: t.numpy().copy() for n, t in grads.items()}, dict(sync.stats), ss, None))  # by value
    except Exception:
        import traceback

        q.put((rank, None, None, None, None, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_c4_tiny_partition_world8_gloo():
    from multimodal_llm_pretraining_amd.params import ALIGN, is_fp32_read
    from multimodal_llm_pretraining_amd.zero3 import Zero3Sync

    # layout at world 8 (every rank lays out the same partition)
    cfg, shapes, st, base = _setup(WORLD, 3)
    thr = 10 * cfg.text.hidden
    assert st.fp32_units == ["text.embed"]
    assert set(st.offsets) == {n for n in shapes if is_fp32_read(n) and math.prod(shapes[n]) <= thr}
    lo = st.fp32_end
    for u, unit in st.units.items():
        assert unit.size % (WORLD * ALIGN) == 0 and unit.shard * WORLD == unit.size, u
        assert unit.local_lo == lo
        lo += unit.shard
    assert lo == st.numel
    order = _order(cfg, st)
    assert order == ["text.embed"] + [f"text.layers.{i}" for i in range(cfg.text.layers)] + \
        ["text.lm_head"]

    # one process accumulating all 16 (rank, micro-batch) contributions
    ref_cfg, _, ref, _ = _setup(1, 0)
    ref.load(base)
    ref.shadow.copy_(ref.master.to(torch.bfloat16))
    rsync = Zero3Sync(ref, _order(ref_cfg, ref))
    assert not _run_micro_batches(ref, rsync, _order(ref_cfg, ref), base,
                                  lambda mb: sum(r + 1 for r in range(WORLD)) * (mb + 1))
    ref.master.copy_(ref.grad)
    want = ref.full_master()
    for n in shapes:  # Σ_r Σ_mb (r+1)(mb+1) = 36 x 3
        assert torch.equal(want[n], base[n] * 108), n

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    L = cfg.text.layers
    n_bf = L + 1  # bf16 units: the layers + lm_head
    for _ in range(WORLD):
        rank, bad, grads, stats, ss, err = q.get(timeout=300)
        assert err is None, err
        assert not bad, (rank, bad[:5])
        for n in shapes:
            assert torch.equal(torch.from_numpy(grads[n]), want[n]), (rank, n)
        # one-unit prefetch, two windows: micro-batch 1 gathers every bf16 unit in forward and
        # all but the two still resident in backward; micro-batch 2 starts with layers 0 and 1
        # resident; the fp32 embedding is gathered once (its window stays bound)
        assert stats["gathers"] == 1 + (2 * n_bf - 2) + (2 * n_bf - 4), stats
        assert stats["reduce_scatters"] == MICRO * (n_bf + 1), stats
        want_ss = sum(float(want[n].double().pow(2).sum()) for n in shapes)
        assert abs(ss - want_ss) <= 1e-6 * want_ss, (ss, want_ss)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0


def test_c4_full_size_layout_world8():
    """Pythia-1B (C4's model) at world 8 on the meta device: the token embedding (103 M
    elements > 10 x 2048) is the one fp32 unit, 16 layers + lm_head are bf16 units, each
    rank holds 1/8 of every unit."""
    from multimodal_llm_pretraining_amd import config as C
    from multimodal_llm_pretraining_amd.params import ALIGN, is_fp32_read
    from multimodal_llm_pretraining_amd.zero3 import Zero3Store

    cfg = C.get_config("pythia-1b")
    shapes = C.param_shapes(cfg)
    st = Zero3Store(shapes, "meta", world=WORLD, rank=7, persist_threshold=10 * cfg.text.hidden)
    assert st.fp32_units == ["text.embed"]
    assert set(st.units) == {"text.embed", "text.lm_head"} | {f"text.layers.{i}" for i in range(16)}
    total = sum(math.prod(s) for s in shapes.values())
    rep = sum(math.prod(s) for n, s in shapes.items() if is_fp32_read(n) and n != "text.embed")
    assert st.fp32_end < rep + 64 * len(shapes)
    part = sum(u.size for u in st.units.values())
    assert total - rep <= part <= total - rep + 2 * WORLD * ALIGN * len(st.units) + 64 * len(shapes)
    assert st.numel == st.fp32_end + part // WORLD
    assert st.numel < 0.13 * total + st.fp32_end  # ~1/8 of the model per rank
