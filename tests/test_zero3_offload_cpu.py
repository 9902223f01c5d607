"""CPU tests of the sharding/offload search space (north star: ZeRO-1/2/3,
activation checkpointing, host offload):

* Zero3Store: the per-unit partition, scatter on load and all-gather of the master;
* Zero3Sync on a world-size-2 gloo group: per-unit gather windows hold the full
  bf16 weights in forward and backward order (prefetch included), gradient windows
  are reduce-scattered (SUM) into each rank's shard, the replicated region is
  all-reduced once per step, Σg² counts the replicated region once;
* libmmpt_host.so (CPU Adam for optimizer offload) against torch.optim.Adam/AdamW.
No HIP compute is called here (the GPU tests run the real engine on these paths).
"""

import math
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _shapes():
    from multimodal_llm_pretraining_amd import config as C

    return C.param_shapes(C.get_config("tiny-mm"))


def _full(shapes, seed=0):
    g = torch.Generator().manual_seed(seed)
    return {n: torch.randn(s, generator=g) for n, s in shapes.items()}


def test_units_cover_every_partitioned_parameter():
    from multimodal_llm_pretraining_amd import config as C
    from multimodal_llm_pretraining_amd.params import ALIGN, is_fp32_read
    from multimodal_llm_pretraining_amd.zero3 import Zero3Store, unit_of

    shapes = _shapes()
    st = Zero3Store(shapes, "cpu", world=3, rank=1)
    seen = set()
    for u, unit in st.units.items():
        assert unit.size % (3 * ALIGN) == 0 and unit.shard * 3 == unit.size
        for n, o in unit.offsets.items():
            assert unit_of(n) == u and o % ALIGN == 0 and o + math.prod(shapes[n]) <= unit.size
            seen.add(n)
    assert seen == {n for n in shapes if not is_fp32_read(n)}
    # the engine's unit order names exactly these units
    cfg = C.get_config("tiny-mm")

    class _E:
        pass

    from multimodal_llm_pretraining_amd.engine import Engine

    e = _E()
    e.cfg, e.s = cfg, st
    assert sorted(Engine.unit_order(e)) == sorted(st.units)
    st_t = Zero3Store(shapes, "cpu", world=3, rank=1, persist_threshold=1000)  # + fp32 units
    e.s = st_t
    assert sorted(Engine.unit_order(e)) == sorted(st_t.units)
    # local layout: replicated region, then one shard per unit, contiguous
    lo = st.fp32_end
    for unit in st.units.values():
        assert unit.local_lo == lo
        lo += unit.shard
    assert lo == st.numel == st.master.numel()


def test_load_scatters_and_single_rank_gather_roundtrips():
    from multimodal_llm_pretraining_amd.zero3 import Zero3Store

    shapes = _shapes()
    full = _full(shapes)
    st = Zero3Store(shapes, "cpu", world=1, rank=0)
    st.load(full)
    back = st.full_master()
    for n in shapes:
        assert torch.equal(back[n], full[n]), n
    with pytest.raises(RuntimeError, match="partitioned"):
        st.p("text.layers.0.qkv.weight")
    with pytest.raises(RuntimeError, match="gathered"):
        st.w("text.layers.0.qkv.weight")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _zero3_worker(rank, world, port, q):
    from multimodal_llm_pretraining_amd.zero3 import Zero3Store, Zero3Sync

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        shapes = _shapes()
        full = _full(shapes)
        st = Zero3Store(shapes, "cpu", world=world, rank=rank)
        st.load(full)
        # every rank holds only its shard; the gather restores the full tensors
        back = st.full_master()
        ok_load = all(torch.equal(back[n], full[n]) for n in shapes)
        st.shadow.copy_(st.master.to(torch.bfloat16))
        order = ["vision.patch"] + [f"vision.layers.{i}" for i in range(2)] + ["proj"] + \
            [f"text.layers.{i}" for i in range(2)] + ["text.lm_head"]
        order = [u for u in order if u in st.units]
        sync = Zero3Sync(st, order)
        bad = []
        for u in order:  # forward
            sync.forward(u)
            for n in st.units[u].offsets:
                if not torch.equal(st.w(n), full[n].to(torch.bfloat16)):
                    bad.append(("fwd", n))
        for u in reversed(order):  # backward: each rank contributes (rank+1) * x
            sync.backward(u)
            for n in st.units[u].offsets:
                if not torch.equal(st.w(n), full[n].to(torch.bfloat16)):
                    bad.append(("bwd", n))
                st.g(n).add_(full[n] * (rank + 1))
            sync.backward_done(u)
        for n in st.offsets:  # replicated region
            st.g(n).add_(full[n] * (rank + 1))
        sync.reduce_grads()
        # Σ over ranks of (r+1)·x = 3x on every shard / the replicated region
        st.master.copy_(st.grad)
        grads = st.full_master()
        ok_grad = all(torch.allclose(grads[n], 3 * full[n], rtol=1e-6, atol=1e-6) for n in shapes)

        class _K:
            @staticmethod
            def sumsq_f32(x, out):
                out.copy_((x.double() ** 2).sum().float().view(1))

        ss = sync.global_sumsq(_K).item()
        want = sum(float((3 * full[n].double()) .pow(2).sum()) for n in shapes)
        q.put((rank, ok_load, bad, ok_grad, ss, want, sync.stats, None))
    except Exception as e:  # report instead of hanging the parent
        import traceback

        q.put((rank, None, None, None, None, None, None, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_zero3_two_rank_gather_and_reduce_scatter():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_zero3_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for _ in range(world):
        rank, ok_load, bad, ok_grad, ss, want, stats, err = q.get(timeout=180)
        assert err is None, err
        assert ok_load and not bad and ok_grad, (rank, bad)
        assert abs(ss - want) <= 1e-5 * want, (ss, want)
        # prefetch: one gather per unit in forward; in backward the last forward unit
        # (lm_head) and the one before it are still resident
        n_units = stats["reduce_scatters"]  # one per unit
        assert n_units == 7  # ViT patch, 2 ViT layers, projector, 2 text layers, lm_head
        assert stats["gathers"] == 2 * n_units - 2, stats
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0


def _zero2_worker(rank, world, port, q):
    from multimodal_llm_pretraining_amd.zero3 import Zero3Store, Zero3Sync

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        shapes = _shapes()
        full = _full(shapes)
        st = Zero3Store(shapes, "cpu", world=world, rank=rank, replicate=True)
        st.load(full)
        st.shadow.copy_(st.master.to(torch.bfloat16))
        order = ["vision.patch"] + [f"vision.layers.{i}" for i in range(2)] + ["proj"] + \
            [f"text.layers.{i}" for i in range(2)] + ["text.lm_head"]
        order = [u for u in order if u in st.units]
        sync = Zero3Sync(st, order)
        bad = []
        # the full bf16 copy is resident from the load on (no gather before the first step)
        for u in order:
            sync.forward(u)
            bad += [("load", n) for n in st.units[u].offsets
                    if not torch.equal(st.w(n), full[n].to(torch.bfloat16))]
        for u in reversed(order):  # gradient path: ZeRO-3's windows + reduce-scatter
            sync.backward(u)
            for n in st.units[u].offsets:
                st.g(n).add_(full[n] * (rank + 1))
            sync.backward_done(u)
        sync.reduce_grads()
        st.master.copy_(st.grad)
        grads = st.full_master()
        ok_grad = all(torch.allclose(grads[n], 3 * full[n], rtol=1e-6, atol=1e-6)
                      for n in shapes if n not in st.offsets)
        # a stand-in update of this rank's shards, then the step's lazy re-gather: every
        # rank sees the full new weights at each unit's first forward, one gather per unit
        st.shadow.copy_((st.master * 0.5).to(torch.bfloat16))
        g0 = sync.stats["gathers"]
        sync.gather_params()
        for u in order:
            sync.forward(u)
            bad += [("step", n) for n in st.units[u].offsets
                    if not torch.equal(st.w(n), (3 * full[n] * 0.5).to(torch.bfloat16))]
        q.put((rank, bad, ok_grad, sync.stats["gathers"] - g0, len(order), None))
    except Exception:
        import traceback

        q.put((rank, None, None, None, None, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_zero2_replicated_weights_partitioned_grads_two_ranks():
    """ZeRO-2 = the ZeRO-3 partition with replicated bf16 weights (DeepSpeed stage 2): no
    full fp32 master / gradient on a rank, gradients reduce-scattered per unit, and after
    a step each unit is all-gathered once, right before its first use."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_zero2_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for _ in range(world):
        rank, bad, ok_grad, gathers, units, err = q.get(timeout=180)
        assert err is None, err
        assert not bad and ok_grad, (rank, bad)
        assert gathers == units
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0


@pytest.mark.parametrize("adamw,wd,clip", [(True, 0.0, None), (True, 0.1, 0.5), (False, 0.01, None)])
def test_host_adam_matches_torch(adamw, wd, clip):
    from multimodal_llm_pretraining_amd.offload import host_adam_step

    n = 4099
    g0 = torch.Generator().manual_seed(3)
    p0 = torch.randn(n, generator=g0)
    p_ref = p0.clone().requires_grad_()
    opt = (torch.optim.AdamW if adamw else torch.optim.Adam)([p_ref], lr=1e-2, betas=(0.9, 0.95),
                                                            eps=1e-8, weight_decay=wd)
    p, m, v = p0.clone(), torch.zeros(n), torch.zeros(n)
    pb = torch.empty(n, dtype=torch.bfloat16)
    for step in range(1, 4):
        g = torch.randn(n, generator=g0)
        p_ref.grad = g * (clip if clip else 1.0)
        opt.step()
        host_adam_step(p, g, m, v, pb, lr=1e-2, beta1=0.9, beta2=0.95, eps=1e-8, weight_decay=wd,
                       adamw=adamw, step=step, grad_scale=clip, threads=2)
        ref = p_ref.detach()
        # torch's foreach/single-tensor kernels order a few ops differently (ulp level,
        # ≪ the lr·1e-6 update scale)
        torch.testing.assert_close(p, ref, rtol=1e-6, atol=1e-7)
        assert torch.equal(pb, p.to(torch.bfloat16))


def test_host_library_exports_header_symbols():
    import re

    from multimodal_llm_pretraining_amd import offload

    src = open(os.path.join(ROOT, "include", "mmpt_host.h")).read()
    syms = sorted(set(re.findall(r"\b(mmpt_host_[a-z0-9_]+)\s*\(", src)))
    assert syms == sorted(offload.HOST_SIGNATURES)
    lib = offload.load_host()
    for s in syms:
        assert hasattr(lib, s)


@pytest.mark.parametrize("adamw,wd", [(True, 0.1), (False, 0.01), (False, 0.0)])
def test_host_adam_vector_clone_bitwise(adamw, wd):
    """The unswitched, vectorised update (AVX-512 or AVX2 clone, whichever this host runs)
    is bitwise the element-wise fp32 sequence of include/mmpt_host.h, evaluated by numpy in
    the same operation order (no contraction), on a ragged length with zeros, tiny values,
    a NaN and an inf in the gradient; bf16 shadow = RNE (a NaN stays a NaN)."""
    import numpy as np

    from multimodal_llm_pretraining_amd.offload import host_adam_step, load_host

    assert load_host().mmpt_host_simd_width() in (8, 16)
    n = 10007
    rng = np.random.default_rng(5)
    p0 = rng.standard_normal(n).astype(np.float32)
    g = rng.standard_normal(n).astype(np.float32)
    g[::97] = 0.0
    g[5::101] = np.float32(1e-38)
    g[7] = np.nan
    g[11] = np.inf
    m0 = (rng.standard_normal(n) * 0.1).astype(np.float32)
    v0 = np.abs(rng.standard_normal(n)).astype(np.float32)
    f = np.float32
    lr, b1, b2, eps, step, sc = f(1e-3), f(0.9), f(0.95), f(1e-8), 3, f(0.5)
    bc1 = 1.0 - float(b1) ** step
    bc2 = 1.0 - float(b2) ** step
    step_size, bc2s = f(float(lr) / bc1), f(np.sqrt(bc2))
    with np.errstate(all="ignore"):
        gr, pi = g * sc, p0.copy()
        if adamw:
            pi = pi * f(f(1.0) - lr * f(wd))
        elif wd != 0.0:
            gr = gr + f(wd) * pi
        mi = m0 + (f(1.0) - b1) * (gr - m0)
        vi = v0 * b2 + (f(1.0) - b2) * gr * gr
        denom = np.sqrt(vi) / bc2s + eps
        pi = pi - step_size * (mi / denom)
    p, m, v = torch.from_numpy(p0.copy()), torch.from_numpy(m0.copy()), torch.from_numpy(v0.copy())
    pb = torch.empty(n, dtype=torch.bfloat16)
    host_adam_step(p, torch.from_numpy(g), m, v, pb, lr=1e-3, beta1=0.9, beta2=0.95, eps=1e-8,
                   weight_decay=wd, adamw=adamw, step=step, grad_scale=0.5, threads=3)
    for got, want in ((p, pi), (m, mi), (v, vi)):
        assert np.array_equal(got.numpy().view(np.uint32), want.astype(np.float32).view(np.uint32))
    fin = torch.isfinite(p) | torch.isinf(p)
    assert torch.equal(pb[fin].view(torch.int16), p[fin].to(torch.bfloat16).view(torch.int16))
    assert torch.isnan(pb[~fin].float()).all()  # NaN stays a (quiet) NaN


@pytest.mark.parametrize("world", [2, 8])
def test_zero2_memory_model_full_size(world):
    """Per-rank fp32 master + gradient bytes of the headline model (ViT-B/16 + Pythia-1B)
    under ZeRO-1 (full buffers: DeepSpeed stage 1 partitions only the optimizer state) and
    ZeRO-2 (DeepSpeed stage 2: master and gradients partitioned; here + the replicated
    fp32-read region and two per-unit gradient windows): laid out on the meta device."""
    from multimodal_llm_pretraining_amd import config as C
    from multimodal_llm_pretraining_amd.params import ParamStore
    from multimodal_llm_pretraining_amd.zero3 import Zero3Store

    shapes = C.param_shapes(C.get_config("vit-b16-pythia-1b"))
    z1 = ParamStore(shapes, "meta", world=world)
    z2 = Zero3Store(shapes, "meta", world=world, rank=0, replicate=True)
    b1 = (z1.master.numel() + z1.grad.numel()) * 4
    b2 = (z2.master.numel() + z2.grad.numel() + sum(w.numel() for w in z2.win_g)) * 4
    # ZeRO-2 keeps the fp32-read region (0.42 B params, mostly the embedding) whole
    assert z2.fp32_end < 0.45e9 and z2.master.numel() < z1.padded / world + z2.fp32_end + 64 * world * 40
    saved = b1 - b2
    assert saved > 0.6 * (1 - 1 / world) * b1 - 8 * z2.fp32_end, (b1, b2)
    print(f"world {world}: ZeRO-1 {b1 / 2**30:.2f} GiB, ZeRO-2 {b2 / 2**30:.2f} GiB fp32 master+grad per rank")


def test_persistence_threshold_layout():
    """DeepSpeed's stage3_param_persistence_threshold: fp32-read parameters at or above it
    (token / position embeddings) become fp32 units — partitioned, laid out right after the
    persistent region ([0, fp32_keep) is what an offload keeps in fp32) — the rest stay
    replicated."""
    from multimodal_llm_pretraining_amd.params import is_fp32_read
    from multimodal_llm_pretraining_amd.zero3 import Zero3Store

    shapes = _shapes()
    thr = 1000
    st = Zero3Store(shapes, "cpu", world=2, rank=1, persist_threshold=thr)
    big = {n for n in shapes if is_fp32_read(n) and math.prod(shapes[n]) > thr}
    assert set(st.fp32_units) == big and {"text.embed", "vision.pos"} <= big
    assert set(st.offsets) == {n for n in shapes if is_fp32_read(n)} - big
    lo = st.fp32_end
    for u in st.fp32_units:
        assert st.units[u].local_lo == lo and st.unit_of(u) == u
        lo += st.units[u].shard
    assert lo == st.fp32_keep
    assert st.win_f32.numel() == max(st.units[u].size for u in st.fp32_units)
    with pytest.raises(RuntimeError, match="gathered"):
        st.p("text.embed")
    with pytest.raises(RuntimeError, match="fp32"):
        st.w("text.embed")


def _f32_unit_worker(rank, world, port, replicate, q):
    from multimodal_llm_pretraining_amd.zero3 import Zero3Store, Zero3Sync

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        shapes = _shapes()
        full = _full(shapes)
        st = Zero3Store(shapes, "cpu", world=world, rank=rank, replicate=replicate,
                        persist_threshold=1000)
        st.load(full)
        st.shadow.copy_(st.master.to(torch.bfloat16))
        f32 = list(st.fp32_units)
        order = ["vision.patch"] + (["vision.pos"] if "vision.pos" in f32 else []) + \
            [f"vision.layers.{i}" for i in range(2)] + ["proj", "text.embed"] + \
            [f"text.layers.{i}" for i in range(2)] + ["text.lm_head"]
        order = [u for u in order if u in st.units]
        sync = Zero3Sync(st, order)
        bad = []
        for step in range(2):
            for u in order:  # forward: the fp32 units in full, exactly
                sync.forward(u)
                if u in f32 and not torch.equal(st.p(u), full[u]):
                    bad.append(("fwd", step, u))
            for u in reversed(order):
                sync.backward(u)
                for n in st.units[u].offsets:
                    st.g(n).copy_(full[n].float() * (rank + 1))
                sync.backward_done(u)
            sync.gather_params()  # (a step: every window / replicated copy stale)
        # two micro-steps of (rank + 1) * x summed over the ranks: 6 x in each rank's shard
        back = {}
        for u in f32:
            unit = st.units[u]
            shard = st.local_shard(st.grad, u)
            flat = torch.zeros(unit.size)
            flat[:full[u].numel()] = full[u].reshape(-1)
            want = 6 * flat[rank * unit.shard:(rank + 1) * unit.shard]
            back[u] = bool(torch.allclose(shard, want, rtol=1e-6, atol=1e-6))
        q.put((rank, bad, back, sync.stats, None))
    except Exception:
        import traceback

        q.put((rank, None, None, None, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("replicate", [False, True])
def test_fp32_units_gather_and_reduce_scatter_gloo_world2(replicate):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_f32_unit_worker, args=(r, world, port, replicate, q))
             for r in range(world)]
    for p in procs:
        p.start()
    for _ in range(world):
        rank, bad, back, stats, err = q.get(timeout=120)
        assert err is None, err
        assert not bad, bad
        assert back and all(back.values()), back
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
