"""ORACLE — test infrastructure only (never imported by the product package).

numpy restatement of the ZeRO++ quantized-communication arithmetic that
`sharding = "zero_3++"` switches on (/root/reference/src/train.py:196-201:
`zero_quantized_weights=True`, `zero_hpz_partition_size=device_count`,
`zero_quantized_gradients=True`).  The algorithm lives in DeepSpeed (the reference's
un-vendored pip dependency, absent from /root/reference and from this image), whose
published ZeRO++ design (qwZ: blockwise symmetric int8 weight all-gather; qgZ: blockwise
int4 gradient all-to-all followed by a local dequantize-and-reduce; hpZ: a secondary
weight partition inside a node) is restated here at the block size the HIP kernels use
(256 elements, one fp32 scale per block, blocks never straddle a rank's shard).
PARITY UNPINNED against DeepSpeed itself (no fixture of its quantized tensors exists in
the reference): the HIP kernels are checked bitwise against this restatement, and the
zero_3++ training step against exact ZeRO-3 and the model oracle within stated bounds.
hpZ is the identity on one node (secondary partition size = GPUs per node = world).
"""

from __future__ import annotations

import numpy as np

QB = 256


def _blocks(n_part: int) -> int:
    return -(-n_part // QB)


def quant_int8(x: np.ndarray, parts: int):
    """bf16-valued fp32 x [parts·n] -> (int8 q [parts·n], fp32 scales [parts·blocks])."""
    x = np.asarray(x, np.float32).reshape(parts, -1)
    n = x.shape[1]
    nb = _blocks(n)
    q = np.zeros_like(x, dtype=np.int8)
    sc = np.zeros((parts, nb), np.float32)
    for r in range(parts):
        for j in range(nb):
            blk = x[r, j * QB:(j + 1) * QB]
            m = np.float32(np.abs(blk).max()) if blk.size else np.float32(0)
            inv = np.float32(127) / m if m > 0 else np.float32(0)
            q[r, j * QB:(j + 1) * QB] = np.clip(np.rint(blk * inv), -127, 127).astype(np.int8)
            sc[r, j] = m / np.float32(127)
    return q.reshape(-1), sc.reshape(-1)


def dequant_int8(q: np.ndarray, sc: np.ndarray, parts: int) -> np.ndarray:
    """-> fp32 values q·scale (the kernel then rounds them to bf16)."""
    q = q.reshape(parts, -1).astype(np.float32)
    n = q.shape[1]
    s = np.repeat(sc.reshape(parts, -1), QB, axis=1)[:, :n]
    return (q * s).reshape(-1)


def quant_int4(x: np.ndarray, parts: int):
    """fp32 x [parts·n] -> (uint8 packed [parts·n/2], fp32 scales [parts·blocks])."""
    x = np.asarray(x, np.float32).reshape(parts, -1)
    n = x.shape[1]
    nb = _blocks(n)
    q = np.zeros_like(x, dtype=np.int8)
    sc = np.zeros((parts, nb), np.float32)
    for r in range(parts):
        for j in range(nb):
            blk = x[r, j * QB:(j + 1) * QB]
            m = np.float32(np.abs(blk).max())
            inv = np.float32(7) / m if m > 0 else np.float32(0)
            q[r, j * QB:(j + 1) * QB] = np.clip(np.rint(blk * inv), -7, 7).astype(np.int8)
            sc[r, j] = m / np.float32(7)
    nib = (q.reshape(-1).astype(np.int16) & 0xF).astype(np.uint8)
    packed = nib[0::2] | (nib[1::2] << 4)
    return packed, sc.reshape(-1)


def unpack_int4(packed: np.ndarray) -> np.ndarray:
    lo = (packed & 0xF).astype(np.int8)
    hi = (packed >> 4).astype(np.int8)
    q = np.empty(packed.size * 2, np.int8)
    q[0::2] = np.where(lo >= 8, lo - 16, lo)
    q[1::2] = np.where(hi >= 8, hi - 16, hi)
    return q


def dequant_int4_sum(packed: np.ndarray, sc: np.ndarray, parts: int) -> np.ndarray:
    """Σ_r q_r·scale_r over the `parts` packed copies of one shard (rank order, fp32)."""
    q = unpack_int4(packed).reshape(parts, -1).astype(np.float32)
    n = q.shape[1]
    s = np.repeat(sc.reshape(parts, -1), QB, axis=1)[:, :n]
    acc = np.zeros(n, np.float32)
    for r in range(parts):
        acc = acc + q[r] * s[r]
    return acc
