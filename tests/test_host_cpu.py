"""CPU-only tests: the C-ABI library loads and exports every symbol
include/mmpt.h declares (no compute calls), host bookkeeping (parameter layout,
label shift / image map, LR schedules vs transformers), and the multi-rank
gradient exchange on a world-size-2 gloo group."""

import os
import re
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "mmpt.h")).read()
    return sorted(set(re.findall(r"\b(mmpt_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree():
    from multimodal_llm_pretraining_amd import _lib

    assert header_symbols() == sorted(_lib.exported_symbols())


def test_library_loads_and_exports_everything():
    from multimodal_llm_pretraining_amd import _lib

    if not os.path.exists(_lib.LIB_PATH):
        import __graft_entry__

        __graft_entry__.build()
    lib = _lib.load()
    for name in header_symbols():
        assert hasattr(lib, name), name
    assert lib.mmpt_abi_version() == _lib.ABI_VERSION
    # size queries are pure host arithmetic
    # δ (fp32 per query row), 256-B aligned, then at D = 256 the dS tiles: ceil(S/32)^2 x 2 KiB
    # per (batch, head)
    delta = -(-(2 * 707 * 8 * 4) // 256) * 256
    assert _lib.query("mmpt_attention_bwd_workspace_bytes", 2, 707, 8, 256) == \
        delta + 2 * 8 * 23 * 23 * 2048
    assert _lib.query("mmpt_attention_bwd_workspace_bytes", 2, 707, 8, 64) == 2 * 707 * 8 * 4
    assert _lib.query("mmpt_layernorm_bwd_workspace_bytes", 4, 64) == 1 * 4 * 64 * 4


def test_kernels_refuse_cpu_tensors():
    from multimodal_llm_pretraining_amd import kernels as K

    a = torch.zeros(8, 8, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="GPU"):
        K.gemm(a, a, torch.zeros(8, 8, dtype=torch.bfloat16))


def test_param_store_layout():
    from multimodal_llm_pretraining_amd import config as C
    from multimodal_llm_pretraining_amd.params import ALIGN, ParamStore

    cfg = C.get_config("tiny-mm")
    st = ParamStore(C.param_shapes(cfg), "cpu", world=3)
    assert st.padded % (3 * ALIGN) == 0 and st.shard_size * 3 == st.padded
    ends = []
    for n, o in st.offsets.items():
        assert o % ALIGN == 0
        ends.append((o, o + st.p(n).numel()))
    ends.sort()
    for (a0, a1), (b0, _) in zip(ends, ends[1:]):
        assert a1 <= b0
    assert C.num_params(cfg) == sum(st.p(n).numel() for n in st.names())


def test_batch_shift_and_image_map():
    from multimodal_llm_pretraining_amd import config as C
    from multimodal_llm_pretraining_amd.engine import Batch

    cfg = C.get_config("tiny-mm")
    npch = cfg.vision.num_patches
    ids = torch.cat([torch.full((2, npch), cfg.image_token_id), torch.randint(0, 1000, (2, 5))], 1)
    labels = ids.clone()
    labels[:, :npch] = -100
    pix = torch.rand(2, 3, cfg.vision.image, cfg.vision.image)
    b = Batch(cfg, ids, labels, pix, torch.device("cpu"))
    lab = b.labels.view(2, -1)
    assert (lab[:, -1] == -100).all()
    assert torch.equal(lab[:, npch - 1:-1], ids[:, npch:])
    assert b.num_items == 2 * 5
    m = b.img_map.view(2, -1)
    assert torch.equal(m[0, :npch], torch.arange(npch, dtype=torch.int32))
    assert torch.equal(m[1, :npch], torch.arange(npch, 2 * npch, dtype=torch.int32))
    assert (m[:, npch:] == -1).all()
    with pytest.raises(ValueError):
        Batch(cfg, ids[:, 1:], labels[:, 1:], pix, torch.device("cpu"))


@pytest.mark.parametrize("kind,kw", [("cosine", {}), ("cosine_with_min_lr", {"min_lr_rate": 0.1}),
                                     ("linear", {}), ("constant", {})])
def test_schedules_match_transformers(kind, kw):
    transformers = pytest.importorskip("transformers")
    from multimodal_llm_pretraining_amd.optim import Schedule

    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.AdamW([p], lr=1e-3)
    sch = transformers.get_scheduler(kind, opt, num_warmup_steps=5, num_training_steps=40,
                                     scheduler_specific_kwargs=kw or None)
    mine = Schedule(1e-3, kind, 5, 40, kw.get("min_lr_rate", 0.0))
    for _ in range(40):
        assert abs(opt.param_groups[0]["lr"] - mine.lr()) < 1e-12
        opt.step()
        sch.step()
        mine.step()


# ------------------------------------------------------------------ gloo world-size 2
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, mode, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from multimodal_llm_pretraining_amd.distributed import GradSync

    n = 4 * 64 * world
    g = torch.arange(n, dtype=torch.float32) * (rank + 1)
    shadow = torch.zeros(n, dtype=torch.bfloat16)
    master = torch.full((n,), float(rank))
    if mode == "ddp_overlap":
        sync = GradSync(g, shadow, n // world, "ddp", min_overlap_elems=1)
        sync.begin_overlap()
        sync.on_ready(n - 100, n)       # e.g. lm_head ready first
        sync.on_ready(64, 200)          # a layer
        sync.on_ready(200, 300)         # the next layer (ranges [0,64) and [300,n-100) never announced)
        mode = "ddp"
    else:
        # fp32-read region [0, fp32_end) spans both shards
        sync = GradSync(g, shadow, n // world, mode, bucket_mb=0.0005, master=master,
                        fp32_end=n // world + 64)
    sync.reduce_grads()
    # a stand-in update on the owned shard (the GPU path runs the fused Adam kernel here)
    if mode == "ddp":
        shadow.copy_(g)
    else:
        sync.shard(shadow).copy_(sync.shard(g))
        sync.shard(master).fill_(100 + rank)
    sync.gather_params()
    q.put((rank, g.numpy().copy(), shadow.float().numpy().copy(), master.numpy().copy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["ddp", "ddp_overlap", "zero1"])
def test_grad_exchange_gloo_world2(mode):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, tuple(map(torch.from_numpy, (g, s, m))))
               for r, g, s, m in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = 4 * 64 * world
    expect = torch.arange(n, dtype=torch.float32) * 3  # Σ_ranks (rank+1) * arange
    for r in range(world):
        g, s, m = res[r]
        if mode in ("ddp", "ddp_overlap"):
            assert torch.equal(g, expect)
        else:
            sh = n // world
            assert torch.equal(g[r * sh:(r + 1) * sh], expect[r * sh:(r + 1) * sh])
            # fp32-read region re-synchronised from its owners; the rest stays local
            assert (m[:sh] == 100).all() and (m[sh:sh + 64] == 101).all()
            assert (m[sh + 64:] == (101 if r == 1 else 0)).all()
        # every rank ends with the full, identical updated parameters
        assert torch.equal(s, expect.to(torch.bfloat16).float())
