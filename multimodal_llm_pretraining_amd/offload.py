"""Optimizer-state offload to host memory (DeepSpeed ZeRO-Offload / FSDP CPUOffload,
selected by the reference's `offloading` knob: experiments/config.py:68-74 →
TrainingClass.zero_offload_optimizer / zero_offload_params / fsdp_offload →
src/train.py:182-213).

The rank's optimizer range (the whole model under DDP, its 1/N shard under ZeRO) keeps
its fp32 master, Adam m and v in pinned host memory; the HBM keeps the bf16 shadow the
step reads, the fp32 gradients and the fp32-read region.  One optimizer step:

  grad shard  --D2H (pinned, copy stream)-->  host
  CPU Adam(W) (libmmpt_host.so, OpenMP, writes fp32 master + bf16 copy)
  bf16 shard  --H2D (second copy stream)-->  HBM shadow;  fp32-read part --H2D--> HBM master

pipelined over 64-MiB chunks: while the host updates chunk i, chunk i+1's gradients are
still coming down and chunk i-1's bf16 parameters going up (PCIe is full duplex), so the
step costs ≈ max(D2H, host Adam, H2D) rather than their sum; the compute stream waits
for the last H2D before the next forward.  Same arithmetic as one whole-range call.

Gradient clipping uses the device Σg² (already reduced across ranks) — the coefficient
is read back once per step.  There is no device fallback: a missing libmmpt_host.so
raises.
"""

from __future__ import annotations

import ctypes
import os
from ctypes import c_double, c_float, c_int, c_int64, c_void_p

import torch

from .optim import AdamConfig

_HERE = os.path.dirname(os.path.abspath(__file__))
HOST_LIB_PATH = os.environ.get("MMPT_HOST_LIB") or os.path.join(_HERE, "lib", "libmmpt_host.so")
HOST_ABI_VERSION = 1

HOST_SIGNATURES = {
    "mmpt_host_abi_version": (c_int, []),
    "mmpt_host_last_error": (ctypes.c_char_p, []),
    "mmpt_host_adam_step": (c_int, [c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_float, c_float, c_float, c_float, c_float, c_int, c_int64,
                                    c_void_p, c_int]),
    "mmpt_host_sumsq": (c_int, [c_int64, c_void_p, ctypes.POINTER(c_double), c_int]),
}

_hlib = None


def load_host() -> ctypes.CDLL:
    global _hlib
    if _hlib is not None:
        return _hlib
    if not os.path.exists(HOST_LIB_PATH):
        raise RuntimeError(f"libmmpt_host.so not found at {HOST_LIB_PATH}: build with "
                           "make -C multimodal_llm_pretraining_amd/csrc")
    lib = ctypes.CDLL(HOST_LIB_PATH)
    for name, (res, args) in HOST_SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    if lib.mmpt_host_abi_version() != HOST_ABI_VERSION:
        raise RuntimeError("libmmpt_host.so ABI mismatch; rebuild")
    _hlib = lib
    return lib


def _host_threads() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))


def host_adam_step(p, g, m, v, pb, *, lr, beta1, beta2, eps, weight_decay, adamw, step,
                   grad_scale=None, threads=0) -> None:
    """CPU Adam(W) over contiguous fp32 CPU tensors (pb: int16/bf16 CPU tensor or None)."""
    lib = load_host()
    for t in (p, g, m, v):
        if t.device.type != "cpu" or t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError("host_adam_step: fp32 contiguous CPU tensors expected")
    gs = None
    if grad_scale is not None:
        gs_t = torch.tensor([float(grad_scale)], dtype=torch.float32)
        gs = gs_t.data_ptr()
    rc = lib.mmpt_host_adam_step(p.numel(), p.data_ptr(), g.data_ptr(), m.data_ptr(),
                                 v.data_ptr(), None if pb is None else pb.data_ptr(), lr, beta1,
                                 beta2, eps, weight_decay, int(adamw), step, gs,
                                 threads or _host_threads())
    if rc != 0:
        raise RuntimeError("mmpt_host_adam_step: " + lib.mmpt_host_last_error().decode())


class HostAdam:
    """FusedAdam's interface (grad_sumsq / step / state_dict) with the optimizer range in
    host memory.  `device_master` + `fp32_end`: the first `fp32_end` elements of this
    rank's range are read by the step from the fp32 master on the device and are copied
    back after each update."""

    def __init__(self, params: torch.Tensor, grads: torch.Tensor, shadow: torch.Tensor | None,
                 cfg: AdamConfig, device_master: torch.Tensor | None = None, fp32_end: int = 0):
        load_host()
        self.dev_p, self.g, self.shadow, self.cfg = params, grads, shadow, cfg
        self.fp32_end = fp32_end
        pin = params.is_cuda
        n = params.numel()
        # the host master is taken from the device master at the first step (so a
        # store.load() after construction is honoured); from then on it is authoritative
        self.p = torch.empty(n, dtype=torch.float32, pin_memory=pin)
        self._initialised = False
        self.m = torch.zeros(n, dtype=torch.float32, pin_memory=pin)
        self.v = torch.zeros(n, dtype=torch.float32, pin_memory=pin)
        self.g_host = torch.empty(n, dtype=torch.float32, pin_memory=pin)
        self.pb_host = torch.empty(n, dtype=torch.bfloat16, pin_memory=pin)
        self.step_count = 0
        self._sumsq = torch.zeros(1, dtype=torch.float32, device=grads.device)
        self._coef = torch.ones(1, dtype=torch.float32, device=grads.device)
        self.chunk = int(os.environ.get("MMPT_OFFLOAD_CHUNK", str(1 << 24)))  # elements
        if self.g.is_cuda:
            self.d2h = torch.cuda.Stream(device=grads.device)
            self.h2d = torch.cuda.Stream(device=grads.device)

    def grad_sumsq(self) -> torch.Tensor:
        from . import kernels as K

        K.sumsq_f32(self.g, self._sumsq)
        return self._sumsq

    def step(self, lr: float, sumsq: torch.Tensor | None = None) -> None:
        from . import kernels as K

        c = self.cfg
        if not self._initialised:
            self.p.copy_(self.dev_p.detach())
            self._initialised = True
        self.step_count += 1
        scale = None
        if c.max_grad_norm and c.max_grad_norm > 0:
            if sumsq is None:
                sumsq = self.grad_sumsq()
            K.clip_coef(sumsq, c.max_grad_norm, self._coef)
            scale = float(self._coef.item())
        kw = dict(lr=lr, beta1=c.betas[0], beta2=c.betas[1], eps=c.eps,
                  weight_decay=c.weight_decay, adamw=c.adamw, step=self.step_count,
                  grad_scale=scale)
        if not self.g.is_cuda:
            self.g_host.copy_(self.g)
            host_adam_step(self.p, self.g_host, self.m, self.v, self.pb_host, **kw)
            if self.shadow is not None:
                self.shadow.copy_(self.pb_host)
            if self.fp32_end:
                self.dev_p[:self.fp32_end].copy_(self.p[:self.fp32_end])
            return
        n = self.p.numel()
        bounds = [(o, min(o + self.chunk, n)) for o in range(0, n, self.chunk)]
        cur = torch.cuda.current_stream(self.g.device)
        self.d2h.wait_stream(cur)  # the gradients (and the clip coefficient) are final
        self.h2d.wait_stream(cur)
        landed = []
        with torch.cuda.stream(self.d2h):
            for lo, hi in bounds:
                self.g_host[lo:hi].copy_(self.g[lo:hi], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.d2h)
                landed.append(ev)
        for (lo, hi), ev in zip(bounds, landed):
            ev.synchronize()
            host_adam_step(self.p[lo:hi], self.g_host[lo:hi], self.m[lo:hi], self.v[lo:hi],
                           self.pb_host[lo:hi], **kw)
            with torch.cuda.stream(self.h2d):
                if self.shadow is not None:
                    self.shadow[lo:hi].copy_(self.pb_host[lo:hi], non_blocking=True)
                f_hi = min(hi, self.fp32_end)
                if f_hi > lo:
                    self.dev_p[lo:f_hi].copy_(self.p[lo:f_hi], non_blocking=True)
        cur.wait_stream(self.h2d)

    def sync_master(self) -> None:
        """Copy the (authoritative) host master of this rank's range back to the device
        master buffer — for checkpoints / inspection, not part of the step."""
        if self._initialised:
            self.dev_p.copy_(self.p)

    def state_dict(self) -> dict:
        return {"m": self.m, "v": self.v, "step": self.step_count}
