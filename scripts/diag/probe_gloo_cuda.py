"""Probe: gloo collectives on CUDA tensors (two ranks sharing cuda:0), default and side stream."""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 1 << 20
    for side in (False, True):
        s = torch.cuda.Stream() if side else torch.cuda.current_stream()
        g = (torch.arange(n, device="cuda", dtype=torch.float32) % 977) * (rank + 1)
        with torch.cuda.stream(s):
            s.wait_stream(torch.cuda.default_stream())
            out = torch.empty(n // world, device="cuda")
            dist.reduce_scatter_tensor(out, g)
            full = torch.empty(n, device="cuda")
            dist.all_gather_into_tensor(full, out)
            ar = g.clone()
            dist.all_reduce(ar)
        torch.cuda.synchronize()
        exp = (torch.arange(n, device="cuda", dtype=torch.float32) % 977) * 3
        print(rank, "side" if side else "default",
              "rs", (out - exp[rank * n // world:(rank + 1) * n // world]).abs().max().item(),
              "ag", (full - exp).abs().max().item(), "ar", (ar - exp).abs().max().item(), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    mp.spawn(worker, args=(2, int(sys.argv[1]) if len(sys.argv) > 1 else 29533), nprocs=2)
