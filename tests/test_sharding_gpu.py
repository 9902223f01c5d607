"""The rest of the reference's sharding / memory search space on the GPU
(training_time_empirical sweep knobs: activation_checkpointing, sharding = zero_3 /
fsdp_full_shard, offloading — experiments/config.py:38-101, src/train.py:126-213):

* activation checkpointing recomputes each layer's forward from its saved input: the
  step is bit-identical to the stored-activation step (same kernels, same inputs);
* ZeRO-3 (per-unit gather / reduce-scatter with prefetch on a side stream): one rank
  alone and two ranks sharing cuda:0 over gloo reproduce one process accumulating the
  same micro-batches — exactly without clipping (fp32 sums in the same order), within
  2 ulp with clipping (Σg² summed as per-rank partials);
* optimizer offload (host Adam in libmmpt_host.so): the master matches the device
  Adam within a few ulp after two steps (the device kernel contracts a·b+c into FMAs,
  the host build does not), the bf16 shadow within one bf16 ulp.
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

NAME, TEXT_LEN = "tiny-mm", 40


def _setup(steps, name=NAME, perturb=False):
    """perturb: weights that differ from init_normal's (a trainer built with init=True holds
    init_normal's weights before load(), so only then does a stale copy show)."""
    from multimodal_llm_pretraining_amd import config as C

    ocfg = oracle_cfg(C.get_config(name))
    P = O.init_params(ocfg, seed=0)
    if perturb:
        g = torch.Generator().manual_seed(7)
        P = {k: v * (1.0 + 0.25 * torch.randn(v.shape, generator=g)) for k, v in P.items()}
    return P, [O.make_batch(ocfg, 4, TEXT_LEN, seed=s) for s in range(1, steps + 1)]


def _trainer(P, sharding="", clip=0.0, ac=False, offload=False, name=NAME):
    from multimodal_llm_pretraining_amd.optim import AdamConfig
    from multimodal_llm_pretraining_amd.trainer import ManualTrainer, StepConfig

    tr = ManualTrainer(StepConfig(model=name, sharding=sharding, scheduler="constant",
                                  activation_checkpointing=ac, offload=offload),
                       AdamConfig(lr=1e-3, max_grad_norm=clip), "cuda")
    tr.store.load(P)
    tr.store.refresh_shadow()
    return tr


def _sl(bd, sl):
    return {k: v[sl] for k, v in bd.items()}


def _run_accumulated(tr, batches):
    """One process: each 4-sample batch as two accumulated 2-sample micro-batches."""
    losses = []
    for bd in batches:
        full = tr.stage(bd)
        mbs = [tr.stage(_sl(bd, slice(0, 2))), tr.stage(_sl(bd, slice(2, 4)))]
        losses.append(tr.train_step(mbs, full.num_items).item() / full.num_items)
    torch.cuda.synchronize()
    return losses


def _master(tr):
    if hasattr(tr.opt, "sync_master"):
        tr.opt.sync_master()
    sd = tr.store.state_dict()
    return {k: v.detach().float().cpu() for k, v in sd.items()}


def test_activation_checkpointing_is_bit_identical():
    P, batches = _setup(2)
    ref = _trainer(P)
    ref_losses = _run_accumulated(ref, batches)
    ac = _trainer(P, ac=True)
    ac_losses = _run_accumulated(ac, batches)
    assert ac_losses == ref_losses
    assert torch.equal(ac.store.master, ref.store.master)
    assert torch.equal(ac.store.shadow, ref.store.shadow)


def test_zero3_single_rank_matches_ddp():
    P, batches = _setup(2)
    ref = _trainer(P)
    ref_losses = _run_accumulated(ref, batches)
    z = _trainer(P, sharding="zero_3")
    z_losses = _run_accumulated(z, batches)
    assert z_losses == ref_losses
    a, b = _master(z), _master(ref)
    for n in b:
        assert torch.equal(a[n], b[n]), n
    assert z.sync.stats["reduce_scatters"] == 2 * 2 * len(z.store.units)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, sharding, clip, ac, offload, steps, q, async_update=None,
            perturb=False):
    import torch.distributed as dist

    if async_update is not None:
        os.environ["MMPT_OFFLOAD_ASYNC"] = "1" if async_update else "0"
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        P, batches = _setup(steps, perturb=perturb)
        tr = _trainer(P, sharding, clip, ac, offload)
        losses = []
        for bd in batches:
            full = tr.stage(bd)
            mine = tr.stage(_sl(bd, slice(2 * rank, 2 * rank + 2)))
            s = tr.train_step([mine], full.num_items).cpu()
            dist.all_reduce(s)
            losses.append(s.item() / full.num_items)
        torch.cuda.synchronize()
        if offload and async_update is not None:
            assert tr.opt.async_update == async_update
        if sharding.startswith(("zero_2", "zero_3")):  # per-unit partition (zero3.py)
            if offload:
                tr.opt.sync_master()  # the host master is authoritative under offload
            m = {k: v.cpu().numpy() for k, v in tr.store.full_master().items()}
        else:
            if offload:
                tr.opt.sync_master()
            lo, hi = rank * tr.store.shard_size, (rank + 1) * tr.store.shard_size
            m = {"__shard__": tr.store.master[lo:hi].cpu().numpy()}
        q.put((rank, losses, m, None))
    except Exception:
        import traceback

        q.put((rank, None, None, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def _two_ranks(sharding, clip, ac, offload, steps, async_update=None, perturb=False):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, sharding, clip, ac, offload, steps, q,
                                               async_update, perturb))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, losses, m, err = q.get(timeout=300)
        assert err is None, err
        # numpy through the queue (torch CPU tensors would travel as shared-memory fds
        # that vanish with the worker)
        res[r] = (losses, {k: torch.from_numpy(v) for k, v in m.items()})
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("clip,ac,steps,exact", [(0.0, False, 2, True), (0.0, True, 2, True),
                                                 (0.5, False, 1, False)])
def test_zero3_two_ranks_match_accumulation(clip, ac, steps, exact):
    res = _two_ranks("zero_3", clip, ac, False, steps)
    P, batches = _setup(steps)
    ref = _trainer(P, clip=clip)
    ref_losses = _run_accumulated(ref, batches)
    want = _master(ref)
    for r, (losses, m) in res.items():
        for a, b in zip(losses, ref_losses):
            assert abs(a - b) < 1e-6, (losses, ref_losses)
        for n, w in want.items():
            d = (m[n] - w).abs()
            if exact:
                assert torch.equal(m[n], w), (r, n, d.max().item())
            else:
                assert (d <= 2.5e-7 * w.abs() + 1e-8).all(), (r, n, d.max().item())


def test_offload_matches_device_adam():
    """One step: master within ulp-level of the device Adam (grads are identical, only the
    update arithmetic differs).  Two steps: loss only — after one step a flipped bf16
    shadow ulp changes the next gradients, and Adam amplifies relative changes of
    gradients near eps to O(lr)."""
    P, batches = _setup(2)
    ref = _trainer(P, clip=0.5)
    off = _trainer(P, clip=0.5, offload=True)
    assert _run_accumulated(off, batches[:1]) == _run_accumulated(ref, batches[:1])
    a, b = _master(off), _master(ref)
    for n in b:
        torch.testing.assert_close(a[n], b[n], rtol=1e-6, atol=2e-8, msg=n)
    sa, sb = off.store.shadow.float(), ref.store.shadow.float()
    assert ((sa - sb).abs() <= 2 ** -7 * sb.abs() + 1e-30).all()
    la, lb = _run_accumulated(off, batches[1:]), _run_accumulated(ref, batches[1:])
    assert abs(la[0] - lb[0]) < 1e-4, (la, lb)


@pytest.mark.parametrize("sharding,name", [("", NAME), ("zero_2", NAME), ("zero_3", NAME),
                                           ("zero_2", "tiny-llama")])
def test_overlapped_offload_is_bit_identical(sharding, name, monkeypatch):
    """Overlapped offload (gradient downloads during the last backward, host Adam on a
    worker thread under the next forward, per-unit gating) against the synchronous update:
    same arithmetic in the same order, so losses and masters are bitwise equal over three
    clipped steps of two accumulated micro-batches — and the overlap really happened.
    tiny-llama: the tied lm_head reads E^T, rebuilt from the persistent region only after
    its host update has landed."""
    P, batches = _setup(3, name)
    monkeypatch.setenv("MMPT_OFFLOAD_ASYNC", "0")
    sync = _trainer(P, sharding, clip=0.5, offload=True, name=name)
    monkeypatch.setenv("MMPT_OFFLOAD_ASYNC", "1")
    over = _trainer(P, sharding, clip=0.5, offload=True, name=name)
    assert over.opt.async_update and not sync.opt.async_update
    la, lb = _run_accumulated(over, batches), _run_accumulated(sync, batches)
    assert la == lb, (la, lb)
    assert over.opt.stats["prefetched_elems"] > 0  # D2H started during the backward
    a, b = _master(over), _master(sync)
    for n in b:
        assert torch.equal(a[n], b[n]), n
    assert torch.equal(over.store.shadow, sync.store.shadow)


@pytest.mark.parametrize("sharding", ["zero_1", "zero_2"])
def test_overlapped_offload_two_ranks_bit_identical(sharding):
    """Two ranks (gloo on cuda:0): the overlapped offload — ZeRO-1's per-chunk shadow
    all-gather gated on the host update (offload.ShardGather), ZeRO-2's per-unit gather
    through the same gate — against the synchronous update: losses and masters bitwise."""
    over = _two_ranks(sharding, 0.5, False, True, 2, async_update=True)
    sync = _two_ranks(sharding, 0.5, False, True, 2, async_update=False)
    for r in range(2):
        (la, ma), (lb, mb) = over[r], sync[r]
        assert la == lb, (r, la, lb)
        assert ma.keys() == mb.keys()
        for k in ma:
            assert torch.equal(ma[k], mb[k]), (r, k)


def test_zero2_offload_two_ranks():
    res = _two_ranks("zero_2", 0.0, False, True, 1)
    P, batches = _setup(1)
    ref = _trainer(P)
    _run_accumulated(ref, batches)
    for r, (losses, m) in res.items():
        for k, v in m.items():  # ZeRO-2 gathers the (host-updated) master by name
            torch.testing.assert_close(torch.as_tensor(v), ref.store.p(k).cpu(), rtol=1e-6,
                                       atol=2e-8)


def test_zero3pp_two_ranks_close_to_exact():
    """zero_3++ (int8 blockwise weight all-gather + int4 gradient all-to-all, 256-element
    blocks; src/train.py:196-201) on two ranks against one exact process over the same
    4-sample batches, clip 1.0, two AdamW steps.  The mode is lossy by design: the step-1
    loss sees int8 weights (relative weight error <= 1/254 per block), the updates see int4
    gradients.  Measured (MI355X): step-1 loss 7.00648 vs exact 7.00714, step-2 7.09772 vs
    7.09911, worst per-tensor update cosine 0.795.  Bounds: step-1 loss within 2e-3, step-2
    within 5e-3, and every tensor's update Δ = master - init points the same way as the
    exact one (cosine > 0.5)."""
    res = _two_ranks("zero_3++", 1.0, False, False, 2)
    P, batches = _setup(2)
    ref = _trainer(P, clip=1.0)
    ref_losses = _run_accumulated(ref, batches)
    want = _master(ref)
    for r, (losses, m) in res.items():
        print(f"rank {r}: zero_3++ {losses} exact {ref_losses}")
        assert abs(losses[0] - ref_losses[0]) < 2e-3, (losses, ref_losses)
        assert abs(losses[1] - ref_losses[1]) < 5e-3, (losses, ref_losses)
        worst = 1.0
        for n, w in want.items():
            d_q, d_x = (m[n] - P[n]).flatten().double(), (w - P[n]).flatten().double()
            if d_x.norm() == 0:
                continue
            cos = float(d_q @ d_x / (d_q.norm() * d_x.norm() + 1e-30))
            worst = min(worst, cos)
            assert cos > 0.5, (n, cos)
        print(f"rank {r}: worst per-tensor update cosine {worst:.3f}")
