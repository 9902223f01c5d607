"""Diagnostic: 2 gloo ranks on cuda:0 (ZeRO or DDP) vs one process (GA over the same two
micro-batches): per-parameter max |Δ| of reduced grads, updated master and bf16 shadow
after ONE optimizer step."""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))


def build(sharding, clip):
    from oracle import model as O
    from test_parity_gpu import oracle_cfg
    from multimodal_llm_pretraining_amd import config as C
    from multimodal_llm_pretraining_amd.optim import AdamConfig
    from multimodal_llm_pretraining_amd.trainer import ManualTrainer, StepConfig

    ocfg = oracle_cfg(C.get_config("tiny-mm"))
    P = O.init_params(ocfg, seed=0)
    bd = O.make_batch(ocfg, 4, 40, seed=1)
    tr = ManualTrainer(StepConfig(model="tiny-mm", sharding=sharding, scheduler="constant"),
                       AdamConfig(lr=1e-3, max_grad_norm=clip), "cuda")
    tr.store.load(P)
    tr.store.refresh_shadow()
    return tr, bd


def one_step(tr, mbs, num_items):
    grads = {}
    orig = tr.sync.reduce_grads

    def rg():
        orig()
        torch.cuda.synchronize()
        grads["g"] = tr.store.grad.clone()
    tr.sync.reduce_grads = rg
    tr.train_step(mbs, num_items)
    torch.cuda.synchronize()
    return grads["g"].cpu(), tr.store.master.cpu(), tr.store.shadow.float().cpu()


def worker(rank, world, port, sharding, clip, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tr, bd = build(sharding, clip)
    full = tr.stage(bd)
    mine = tr.stage({k: v[2 * rank:2 * rank + 2] for k, v in bd.items()})
    g, m, s = one_step(tr, [mine], full.num_items)
    q.put((rank, g.numpy(), m.numpy(), s.numpy(), dict(tr.store.offsets), tr.store.shard_size))
    dist.destroy_process_group()


if __name__ == "__main__":
    sharding = sys.argv[1] if len(sys.argv) > 1 else "zero_1"
    clip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, 2, 29611, sharding, clip, q)) for r in range(2)]
    [p.start() for p in ps]
    res = {}
    for _ in range(2):
        r, *rest = q.get(timeout=300)
        res[r] = [torch.from_numpy(x) if hasattr(x, 'dtype') else x for x in rest]
    [p.join() for p in ps]
    tr, bd = build("", clip)
    full = tr.stage(bd)
    mbs = [tr.stage({k: v[0:2] for k, v in bd.items()}), tr.stage({k: v[2:4] for k, v in bd.items()})]
    g0, m0, s0 = one_step(tr, mbs, full.num_items)
    print(f"mode={sharding} clip={clip}")
    for name, off in tr.store.offsets.items():
        n = tr.store.p(name).numel()
        worst = {"g": 0.0, "m": 0.0, "s": 0.0}
        for r in range(2):
            g, m, s, offs, sh = res[r]
            o = offs[name]
            lo, hi = max(o, r * sh), min(o + n, (r + 1) * sh)
            if sharding == "":
                lo, hi = o, o + n
            if hi > lo:
                ref_lo = lo - o + off
                worst["g"] = max(worst["g"], (g[lo:hi] - g0[ref_lo:ref_lo + hi - lo]).abs().max().item())
                worst["m"] = max(worst["m"], (m[lo:hi] - m0[ref_lo:ref_lo + hi - lo]).abs().max().item())
            worst["s"] = max(worst["s"], (s[o:o + n] - s0[off:off + n]).abs().max().item())
        if max(worst.values()) > 0:
            print(f"{name:32s} off={off:8d} n={n:8d} dg={worst['g']:.3e} dm={worst['m']:.3e} ds={worst['s']:.3e}")
    print("done", flush=True)
