"""Thin tensor-level wrappers over the libmmpt C-ABI (include/mmpt.h).

PyTorch is used only as plumbing here: device memory (the caching allocator),
the current HIP stream and shape bookkeeping.  Every arithmetic operation is a
call into the hand-written HIP library; nothing falls back to ATen.
"""

from __future__ import annotations

import torch

from . import _lib

ROWS_K, K_ROWS = 0, 1
EPI_BF16, EPI_BF16_GELU, EPI_BF16_DGELU, EPI_F32_ACC, EPI_F32_STORE, EPI_F32_RESID, EPI_BF16_DGELU_COLSUM = range(7)
# quick-GELU (CLIP) forms of the GELU epilogues
EPI_BF16_QGELU, EPI_BF16_DQGELU, EPI_BF16_DQGELU_COLSUM = 7, 8, 9
# SwiGLU (Llama MLP) with the gate|up projection in 128-column blocks (include/mmpt.h)
EPI_BF16_SWIGLU, EPI_BF16_DSWIGLU = 10, 11
EPI_F32_ACC_COLSUM = 12

_ws_cache: dict[tuple[int, int, int], torch.Tensor] = {}

# Optional live instrumentation (bench.py roofline): when set, every GEMM launch is
# bracketed by HIP events on its own stream and its algorithmic FLOPs recorded.
_gemm_probe: list | None = None


def start_gemm_probe() -> None:
    global _gemm_probe
    _gemm_probe = []


def stop_gemm_probe() -> list:
    """Returns [(kernel_name, flops, algorithmic_bytes, start_event, end_event, shape,
    stream), ...] (end_event = end of the main GEMM kernel; shape = (M, N, K, epilogue);
    stream = the HIP stream the launch went to); caller synchronizes."""
    global _gemm_probe
    out, _gemm_probe = _gemm_probe or [], None
    return out


def gemm_kernel_name(M: int, N: int, K: int, layout_a: int, layout_b: int, epilogue: int,
                     workspace_bytes: int) -> str:
    """The exact kernel (as rocprofv3 names it) mmpt_gemm_bf16 launches for this problem."""
    import ctypes

    buf = ctypes.create_string_buffer(64)
    _lib.call("mmpt_gemm_kernel_name", layout_a, layout_b, epilogue, M, N, K, workspace_bytes,
              buf, 64)
    return buf.value.decode()


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _p(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def workspace(nbytes: int, slot: int = 0, device: torch.device | None = None) -> torch.Tensor:
    """Persistent scratch per (device, slot, stream): kernels running concurrently on
    different streams (Engine's weight-gradient stream) never share a workspace."""
    dev = torch.cuda.current_device() if device is None else device.index
    key = (dev, slot, torch.cuda.current_stream(dev).cuda_stream)
    ws = _ws_cache.get(key)
    if ws is None or ws.numel() < nbytes:
        ws = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=f"cuda:{dev}")
        _ws_cache[key] = ws
    return ws


def _check(t: torch.Tensor, dtype: torch.dtype, name: str) -> None:
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_cuda:
        raise RuntimeError(f"{name}: tensor must live on the GPU (no CPU fallback)")


def _ld(t: torch.Tensor) -> int:
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError("expected a 2-D tensor with unit inner stride")
    return t.stride(0)


# ----------------------------------------------------------------------------- GEMM
def gemm(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, *, layout_a: int = ROWS_K,
         layout_b: int = ROWS_K, epilogue: int = EPI_BF16, bias: torch.Tensor | None = None,
         aux: torch.Tensor | None = None, out2: torch.Tensor | None = None) -> torch.Tensor:
    """out = op(a) @ op(b) with a fused epilogue (see include/mmpt.h mmpt_epilogue).

    layout ROWS_K: operand stored [rows][K]; K_ROWS: stored [K][rows].
    """
    _check(a, torch.bfloat16, "gemm.a")
    _check(b, torch.bfloat16, "gemm.b")
    if layout_a == ROWS_K:
        M, K = a.shape
    else:
        K, M = a.shape
    if layout_b == ROWS_K:
        N, Kb = b.shape
    else:
        Kb, N = b.shape
    if K != Kb:
        raise ValueError(f"gemm: K mismatch {K} vs {Kb}")
    want = (M, 2 * N) if epilogue == EPI_BF16_DSWIGLU else (M, N)  # dgate|dup, blocked
    if tuple(out.shape) != want:
        raise ValueError(f"gemm: out shape {tuple(out.shape)} != {want}")
    if epilogue == EPI_BF16_SWIGLU and (out2 is None or tuple(out2.shape) != (M, N // 2)):
        raise ValueError("gemm: SWIGLU needs out2 [M, N/2] (the activation)")
    if epilogue == EPI_BF16_DSWIGLU and (aux is None or tuple(aux.shape) != (M, 2 * N)):
        raise ValueError("gemm: DSWIGLU needs aux [M, 2N] (the forward's gate|up)")
    wsb = _lib.query("mmpt_gemm_workspace_bytes", M, N, K, epilogue)
    ws = workspace(wsb, slot=5) if wsb > 0 else None
    probe = _gemm_probe
    if probe is not None:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev1.record()  # materialise the hipEvent; re-recorded by the library after the main kernel
        ev0.record()
        _lib.load().mmpt_gemm_probe_event(ev1.cuda_event)
    _lib.call(
        "mmpt_gemm_bf16", layout_a, layout_b, epilogue, M, N, K,
        a.data_ptr(), _ld(a), b.data_ptr(), _ld(b), out.data_ptr(), _ld(out),
        _p(bias), _p(aux), 0 if aux is None else _ld(aux),
        _p(out2), 0 if out2 is None else _ld(out2), _p(ws), wsb, _stream(),
    )
    if probe is not None:
        out_b = {EPI_BF16: 2, EPI_BF16_GELU: 4, EPI_BF16_DGELU: 4, EPI_F32_ACC: 8,
                 EPI_F32_STORE: 4, EPI_F32_RESID: 10, EPI_BF16_DGELU_COLSUM: 4,
                 EPI_BF16_QGELU: 4, EPI_BF16_DQGELU: 4, EPI_BF16_DQGELU_COLSUM: 4,
                 EPI_BF16_SWIGLU: 3, EPI_BF16_DSWIGLU: 8, EPI_F32_ACC_COLSUM: 8}[epilogue]
        import ctypes

        name = ctypes.create_string_buffer(64)  # the launch's own choice (alignment included)
        _lib.call("mmpt_gemm_last_kernel_name", name, 64)
        mt = _lib.query("mmpt_gemm_last_tail_rows")  # rows computed by the tail split (if any)
        mm = M - mt
        st = _stream()
        probe.append((name.value.decode(),
                      2.0 * mm * N * K, 2.0 * (mm + N) * K + out_b * mm * N, ev0, ev1,
                      (mm, N, K, epilogue), st))
        if mt > 0:  # the tail: split-K launch + epilogue kernel, from the main launch's end
            ev2 = torch.cuda.Event(enable_timing=True)
            ev2.record()
            probe.append((f"gemm4p_kernel<{layout_a}, {layout_b}, 100>+tail_epi_kernel",
                          2.0 * mt * N * K, 2.0 * (mt + N) * K + out_b * mt * N, ev1, ev2,
                          (mt, N, K, epilogue), st))
    return out


def gemm_last_kernel() -> str:
    """The kernel (with its template arguments) this thread's last `gemm` launched."""
    import ctypes

    name = ctypes.create_string_buffer(64)
    _lib.call("mmpt_gemm_last_kernel_name", name, 64)
    return name.value.decode()


def gemm_dgelu_colsum(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, pre: torch.Tensor,
                      dbias: torch.Tensor, quick: bool = False) -> torch.Tensor:
    """out = bf16(bf16(a @ b^T) * gelu'(pre)) and dbias += bf16(Σ_rows out) — the fc1 input
    gradient and fc1 bias gradient in one GEMM pass (per-tile column sums in the epilogue,
    then a fixed-order reduce)."""
    M, N = out.shape
    rows = _lib.query("mmpt_gemm_colsum_rows", M, N, a.shape[1])
    part = workspace(rows * N * 4, slot=6).view(torch.float32)[: rows * N]
    gemm(a, b, out, epilogue=EPI_BF16_DQGELU_COLSUM if quick else EPI_BF16_DGELU_COLSUM, aux=pre,
         out2=part.view(rows, N))
    _lib.call("mmpt_colsum_f32", rows, N, part.data_ptr(), dbias.data_ptr(), None, 1, _stream())
    return out


def gemm_wgrad_colsum(dy: torch.Tensor, x: torch.Tensor, dw: torch.Tensor, dbias: torch.Tensor,
                      dbias2: torch.Tensor | None = None) -> bool:
    """dw += dyᵀ·x (fp32) and dbias (and dbias2) += bf16(Σ_rows dy) in one GEMM pass
    (EPI_F32_ACC_COLSUM: the weight-gradient GEMM sums the dy fragments its MFMAs read, one
    partial row per K split, then a fixed-order reduce) — addmm backward's grad_weight and
    grad_bias without a second read of dy.  Returns False, having done nothing, when the fused
    form does not take the problem (mmpt_gemm_acc_colsum_rows == 0): use gemm + colsum."""
    T, M = dy.shape
    N = x.shape[1]
    rows = _lib.query("mmpt_gemm_acc_colsum_rows", M, N, T)
    if rows <= 0:
        return False
    part = workspace(rows * M * 4, slot=8).view(torch.float32)[: rows * M].view(rows, M)
    gemm(dy, x, dw, layout_a=K_ROWS, layout_b=K_ROWS, epilogue=EPI_F32_ACC_COLSUM, out2=part)
    _lib.call("mmpt_colsum_f32", rows, M, part.data_ptr(), dbias.data_ptr(), _p(dbias2), 1,
              _stream())
    return True


def colsum(dy: torch.Tensor, dbias: torch.Tensor, accumulate: bool = True,
           dbias2: torch.Tensor | None = None) -> None:
    rows, cols = dy.shape
    ws = workspace(_lib.query("mmpt_colsum_workspace_bytes", rows, cols), slot=1)
    _lib.call("mmpt_colsum_bf16", rows, cols, dy.data_ptr(), _ld(dy), dbias.data_ptr(),
              _p(dbias2), int(accumulate), ws.data_ptr(), _stream())


# ----------------------------------------------------------------------------- LayerNorm
def layernorm_fwd(x: torch.Tensor, w1, b1, eps: float, y1: torch.Tensor, mean: torch.Tensor,
                  rstd: torch.Tensor, w2=None, b2=None, y2: torch.Tensor | None = None) -> None:
    _check(x, torch.float32, "layernorm.x")
    rows, h = x.shape
    _lib.call("mmpt_layernorm_fwd", rows, h, float(eps), x.data_ptr(), _ld(x), w1.data_ptr(),
              b1.data_ptr(), y1.data_ptr(), _p(w2), _p(b2), _p(y2), mean.data_ptr(),
              rstd.data_ptr(), _stream())


def layernorm_bwd(x, mean, rstd, dy1, w1, dx, dw1, db1, dy2=None, w2=None, dw2=None, db2=None,
                  dresid=None, dx_bf16=None, dsum=None, dsum2=None) -> None:
    """dx = dresid + LN'(dy1) (+ LN'(dy2)); dγ/dβ += ...; optionally dx_bf16 = bf16(dx) and
    dsum (+ dsum2) += bf16(Σ_rows bf16(dx)) (fused cast + bias-gradient column sum)."""
    rows, h = x.shape
    ws = workspace(_lib.query("mmpt_layernorm_bwd_ex_workspace_bytes", rows, h), slot=2)
    _lib.call("mmpt_layernorm_bwd_ex", rows, h, x.data_ptr(), _ld(x), mean.data_ptr(),
              rstd.data_ptr(), dy1.data_ptr(), w1.data_ptr(), _p(dy2), _p(w2), _p(dresid),
              dx.data_ptr(), _p(dx_bf16), _p(dw1), _p(db1), _p(dw2), _p(db2), _p(dsum),
              _p(dsum2), ws.data_ptr(), _stream())


def layernorm_f32_fwd(x, w, b, eps: float, y, mean, rstd) -> None:
    _check(x, torch.float32, "layernorm_f32.x")
    rows, h = x.shape
    _lib.call("mmpt_layernorm_f32_fwd", rows, h, float(eps), x.data_ptr(), w.data_ptr(),
              b.data_ptr(), y.data_ptr(), mean.data_ptr(), rstd.data_ptr(), _stream())


def layernorm_f32_bwd(x, mean, rstd, dy, w, dx, dw, db) -> None:
    rows, h = x.shape
    ws = workspace(_lib.query("mmpt_layernorm_bwd_workspace_bytes", rows, h), slot=2)
    _lib.call("mmpt_layernorm_f32_bwd", rows, h, x.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
              dy.data_ptr(), w.data_ptr(), dx.data_ptr(), _p(dw), _p(db), ws.data_ptr(),
              _stream())


# ----------------------------------------------------------------------------- attention
def rope_inplace(qkv: torch.Tensor, seq: int, heads: int, head_dim: int, rot_dims: int,
                 head_stride: int, part_stride: int, cos: torch.Tensor, sin: torch.Tensor,
                 inverse: bool = False, parts: int = 2, offset: int = 0) -> None:
    """Rotate `parts` (2: q and k at part_stride apart; 1: one of them) of `heads` heads
    starting `offset` elements into each qkv row."""
    tokens = qkv.shape[0]
    _lib.call("mmpt_rope_inplace", tokens, seq, heads, head_dim, rot_dims,
              qkv.data_ptr() + offset * qkv.element_size(), _ld(qkv), head_stride, part_stride,
              parts, cos.data_ptr(), sin.data_ptr(), int(inverse), _stream())


def rmsnorm_fwd(x: torch.Tensor, w, eps: float, y: torch.Tensor, rstd: torch.Tensor) -> None:
    _check(x, torch.float32, "rmsnorm.x")
    rows, h = x.shape
    _lib.call("mmpt_rmsnorm_fwd", rows, h, float(eps), x.data_ptr(), _ld(x), w.data_ptr(),
              y.data_ptr(), rstd.data_ptr(), _stream())


def rmsnorm_bwd(x, rstd, dy, w, dx, dw=None, dresid=None, dx_bf16=None) -> None:
    """dx = dresid + RMS'(dy; w) (dx may alias dresid); dw += Σ dy·x̂; optional bf16 copy."""
    rows, h = x.shape
    ws = workspace(_lib.query("mmpt_rmsnorm_bwd_workspace_bytes", rows, h), slot=2)
    _lib.call("mmpt_rmsnorm_bwd", rows, h, x.data_ptr(), _ld(x), rstd.data_ptr(), dy.data_ptr(),
              w.data_ptr(), _p(dresid), dx.data_ptr(), _p(dx_bf16), _p(dw), ws.data_ptr(), _stream())


def attention_fwd(qkv, batch, seq, heads, head_dim, head_stride, part_stride, causal, scale,
                  out, lse) -> None:
    _lib.call("mmpt_attention_fwd", batch, seq, heads, head_dim, qkv.data_ptr(), _ld(qkv),
              head_stride, part_stride, int(causal), float(scale), out.data_ptr(), _ld(out),
              lse.data_ptr(), _stream())


def attention_bwd(qkv, batch, seq, heads, head_dim, head_stride, part_stride, causal, scale,
                  out, dout, lse, dqkv) -> None:
    ws = workspace(_lib.query("mmpt_attention_bwd_workspace_bytes", batch, seq, heads, head_dim),
                   slot=3)
    _lib.call("mmpt_attention_bwd", batch, seq, heads, head_dim, qkv.data_ptr(), _ld(qkv),
              head_stride, part_stride, int(causal), float(scale), out.data_ptr(),
              dout.data_ptr(), _ld(out), lse.data_ptr(), dqkv.data_ptr(), ws.data_ptr(),
              _stream())


def attention_bwd_rope(qkv, batch, seq, heads, head_dim, head_stride, part_stride, causal, scale,
                       out, dout, lse, dqkv, rot_dims, cos, sin) -> None:
    """attention_bwd + rope_inplace(dqkv, inverse=True) on the q and k parts (one kernel pass
    less at head_dim 256 / 64 rotary dims: the dK / dQ epilogues rotate)."""
    ws = workspace(_lib.query("mmpt_attention_bwd_workspace_bytes", batch, seq, heads, head_dim),
                   slot=3)
    _lib.call("mmpt_attention_bwd_rope", batch, seq, heads, head_dim, qkv.data_ptr(), _ld(qkv),
              head_stride, part_stride, int(causal), float(scale), out.data_ptr(),
              dout.data_ptr(), _ld(out), lse.data_ptr(), dqkv.data_ptr(), ws.data_ptr(),
              rot_dims, cos.data_ptr(), sin.data_ptr(), _stream())


def attention_gqa_fwd(qkv, batch, seq, heads, kv_heads, head_dim, k_offset, v_offset, causal,
                      scale, out, lse) -> None:
    """Llama GQA: q head h at h*head_dim, its kv head h // (heads/kv_heads) at
    k_offset / v_offset + j*head_dim of each fused-qkv row."""
    _lib.call("mmpt_attention_gqa_fwd", batch, seq, heads, kv_heads, head_dim, qkv.data_ptr(),
              _ld(qkv), head_dim, k_offset, v_offset, int(causal), float(scale), out.data_ptr(),
              _ld(out), lse.data_ptr(), _stream())


def attention_gqa_bwd(qkv, batch, seq, heads, kv_heads, head_dim, k_offset, v_offset, causal,
                      scale, out, dout, lse, dqkv) -> None:
    ws = workspace(_lib.query("mmpt_attention_bwd_workspace_bytes", batch, seq, heads, head_dim),
                   slot=3)
    _lib.call("mmpt_attention_gqa_bwd", batch, seq, heads, kv_heads, head_dim, qkv.data_ptr(),
              _ld(qkv), head_dim, k_offset, v_offset, int(causal), float(scale), out.data_ptr(),
              dout.data_ptr(), _ld(out), lse.data_ptr(), dqkv.data_ptr(), ws.data_ptr(), _stream())


# ----------------------------------------------------------------------------- loss
def cross_entropy(logits, labels, ignore_index: int, grad_scale: float, loss_rows,
                  dlogits=None, vocab_valid: int | None = None) -> None:
    """vocab_valid: logit columns past it are padding (excluded, zero gradient)."""
    rows, vocab = logits.shape
    _lib.call("mmpt_cross_entropy", rows, vocab, vocab_valid or vocab, logits.data_ptr(), _ld(logits),
              labels.data_ptr(), ignore_index, float(grad_scale), loss_rows.data_ptr(),
              _p(dlogits), 0 if dlogits is None else _ld(dlogits), _stream())


def sum_f32(x: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    n = x.numel()
    ws = workspace(_lib.query("mmpt_sum_workspace_bytes", n), slot=4)
    _lib.call("mmpt_sum_f32", n, x.data_ptr(), out.data_ptr(), ws.data_ptr(), _stream())
    return out


def sumsq_f32(x: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    n = x.numel()
    ws = workspace(_lib.query("mmpt_l2norm_workspace_bytes", n), slot=4)
    _lib.call("mmpt_sumsq_f32", n, x.data_ptr(), out.data_ptr(), ws.data_ptr(), _stream())
    return out


# ----------------------------------------------------------------------------- ZeRO++ quantization
QUANT_BLOCK = 256


def quant_blocks(n_part: int) -> int:
    """fp32 scales per part of n_part elements (256-element blocks, the last one partial)."""
    return -(-n_part // QUANT_BLOCK)


def _quant_args(n_part, parts, *tensors):
    if n_part <= 0 or n_part % 4:
        raise ValueError(f"quantization part of {n_part} elements (need a positive multiple of 4)")
    for t in tensors:
        if not t.is_contiguous():
            raise ValueError("quantization buffers must be contiguous")


def quant_int8(src: torch.Tensor, parts: int, dst: torch.Tensor, scales: torch.Tensor) -> None:
    """bf16 [parts·n] -> int8 [parts·n] + fp32 scales [parts·blocks] (qwZ)."""
    _check(src, torch.bfloat16, "src")
    n = src.numel() // parts
    _quant_args(n, parts, src, dst, scales)
    if dst.dtype != torch.int8 or dst.numel() < parts * n or scales.numel() < parts * quant_blocks(n):
        raise ValueError("quant_int8: dst int8 / scales too small")
    _lib.call("mmpt_quant_int8", n, parts, src.data_ptr(), dst.data_ptr(), scales.data_ptr(), _stream())


def dequant_int8(src: torch.Tensor, scales: torch.Tensor, parts: int, dst: torch.Tensor) -> None:
    _check(dst, torch.bfloat16, "dst")
    n = dst.numel() // parts
    _quant_args(n, parts, src, dst, scales)
    if src.dtype != torch.int8 or src.numel() < parts * n or scales.numel() < parts * quant_blocks(n):
        raise ValueError("dequant_int8: src int8 / scales too small")
    _lib.call("mmpt_dequant_int8", n, parts, src.data_ptr(), scales.data_ptr(), dst.data_ptr(), _stream())


def quant_int4(src: torch.Tensor, parts: int, dst: torch.Tensor, scales: torch.Tensor) -> None:
    """fp32 [parts·n] -> packed int4 uint8 [parts·n/2] + fp32 scales [parts·blocks] (qgZ)."""
    _check(src, torch.float32, "src")
    n = src.numel() // parts
    _quant_args(n, parts, src, dst, scales)
    if dst.dtype != torch.uint8 or dst.numel() < parts * n // 2 or scales.numel() < parts * quant_blocks(n):
        raise ValueError("quant_int4: dst uint8 / scales too small")
    _lib.call("mmpt_quant_int4", n, parts, src.data_ptr(), dst.data_ptr(), scales.data_ptr(), _stream())


def dequant_int4_sum(src: torch.Tensor, scales: torch.Tensor, parts: int, dst: torch.Tensor) -> None:
    """dst (fp32, n) += Σ over the `parts` packed int4 copies of it in src (rank order)."""
    _check(dst, torch.float32, "dst")
    n = dst.numel()
    _quant_args(n, parts, src, dst, scales)
    if src.dtype != torch.uint8 or src.numel() < parts * n // 2 or scales.numel() < parts * quant_blocks(n):
        raise ValueError("dequant_int4_sum: src uint8 / scales too small")
    _lib.call("mmpt_dequant_int4_sum", n, parts, src.data_ptr(), scales.data_ptr(), dst.data_ptr(),
              _stream())


# ----------------------------------------------------------------------------- embeddings
def gather_rows(src, idx, dst) -> None:
    _lib.call("mmpt_gather_rows_bf16", dst.shape[0], dst.shape[1], _p(idx), src.data_ptr(),
              _ld(src), dst.data_ptr(), _ld(dst), _stream())


def expand_rows(src, row_map, dst) -> None:
    _lib.call("mmpt_expand_rows_bf16", dst.shape[0], dst.shape[1], row_map.data_ptr(),
              src.data_ptr(), _ld(src), dst.data_ptr(), _ld(dst), _stream())


def embed_fwd(ids, table, out, img_map=None, img=None) -> None:
    rows, h = out.shape
    _lib.call("mmpt_embed_fwd", rows, h, ids.data_ptr(), table.data_ptr(), _p(img_map), _p(img),
              out.data_ptr(), _stream())


def embed_segments(ids, vocab: int, skip_id: int = -1):
    """The deterministic embedding-backward order built on the device (mmpt_embed_segments):
    returns (seg_id, seg_off, perm, nseg, bad) int32 device tensors — the text rows (id !=
    skip_id) stably sorted by id, one segment per distinct id, the segment count `nseg` [1]
    and the out-of-range flag `bad` [1] left in device memory (no host synchronisation)."""
    _check(ids, torch.int64, "embed_segments ids")
    rows = ids.numel()
    dev = ids.device
    out = torch.empty(3 * rows + 3, dtype=torch.int32, device=dev)
    seg_id, seg_off = out[:rows], out[rows:2 * rows + 1]
    perm, nseg, bad = out[2 * rows + 1:3 * rows + 1], out[3 * rows + 1:3 * rows + 2], out[3 * rows + 2:]
    wsb = _lib.query("mmpt_embed_segments_workspace_bytes", rows, vocab)
    if wsb < 0:
        raise ValueError(f"embed_segments: unsupported sizes rows={rows} vocab={vocab}")
    ws = workspace(wsb, slot=7, device=dev)
    _lib.call("mmpt_embed_segments", rows, ids.data_ptr(), vocab, skip_id, seg_id.data_ptr(),
              seg_off.data_ptr(), perm.data_ptr(), nseg.data_ptr(), bad.data_ptr(), ws.data_ptr(),
              ws.numel(), _stream())
    return seg_id, seg_off, perm, nseg, bad


def embed_bwd(segments, dout, dtable=None, img_map=None, dimg=None) -> None:
    """segments = (seg_id, seg_off, perm[, nseg, bad]) int32 device tensors: the text rows
    sorted by token id (engine.Batch.segments) — the deterministic scatter-add order.  With
    the device segment count (embed_segments) the kernel reads nseg from HBM."""
    rows, h = dout.shape
    if len(segments) >= 4:
        # device segments (embed_segments): segments longer than 1024 rows are summed over
        # 256-row chunks of the sorted order, then the chunk sums in order (mmpt_embed_bwd_split)
        seg_id, seg_off, perm, nseg = segments[:4]
        n = perm.numel()
        wsb = _lib.query("mmpt_embed_bwd_split_workspace_bytes", max(n, 1), h)
        ws = workspace(wsb, slot=9, device=dout.device) if dtable is not None and n else None
        _lib.call("mmpt_embed_bwd_split", rows, h, n, nseg.data_ptr(), _p(seg_id),
                  _p(seg_off), _p(perm), _p(img_map), dout.data_ptr(), _p(dtable), _p(dimg),
                  _p(ws), 0 if ws is None else ws.numel(), _stream())
        return
    seg_id, seg_off, perm = segments
    _lib.call("mmpt_embed_bwd", rows, h, seg_id.numel(), _p(seg_id), _p(seg_off), _p(perm),
              _p(img_map), dout.data_ptr(), _p(dtable), _p(dimg), _stream())


def im2col(pixels, patch, cols) -> None:
    b, c, s, _ = pixels.shape
    if patch % 8 == 0 and cols.shape[1] == c * patch * patch:
        _lib.call("mmpt_im2col_patches", b, c, s, patch, pixels.data_ptr(), cols.data_ptr(),
                  _stream())
    else:  # CLIP-L/14 etc.: padded K
        _lib.call("mmpt_im2col_patches_ex", b, c, s, patch, pixels.data_ptr(), cols.data_ptr(),
                  _ld(cols), _stream())


def vit_embed_fwd(batch, num_patches, patch_out, cls, pos, out) -> None:
    h = patch_out.shape[-1]
    _lib.call("mmpt_vit_embed_fwd", batch, num_patches, h, patch_out.data_ptr(), cls.data_ptr(),
              pos.data_ptr(), out.data_ptr(), _stream())


def vit_embed_bwd(batch, num_patches, dout, dcls, dpos, dpatch) -> None:
    h = dout.shape[-1]
    _lib.call("mmpt_vit_embed_bwd", batch, num_patches, h, dout.data_ptr(), _p(dcls), _p(dpos),
              _p(dpatch), _stream())


def select_patches_fwd(batch, num_patches, x, out) -> None:
    _lib.call("mmpt_select_patches_fwd", batch, num_patches, x.shape[-1], x.data_ptr(),
              out.data_ptr(), _stream())


def select_patches_bwd(batch, num_patches, dout, dx, accumulate: bool) -> None:
    _lib.call("mmpt_select_patches_bwd", batch, num_patches, dx.shape[-1], dout.data_ptr(),
              dx.data_ptr(), int(accumulate), _stream())


# ----------------------------------------------------------------------------- optimizer
def adam_step(param, grad, exp_avg, exp_avg_sq, param_bf16, *, lr, beta1, beta2, eps,
              weight_decay, adamw: bool, step: int, grad_scale=None, zero_grad: bool = False,
              max_blocks: int = 0) -> None:
    """zero_grad: the kernel also zeroes `grad` as it consumes it (mmpt_adam_step_zero_grad,
    whose grid max_blocks > 0 caps)."""
    args = [param.numel(), param.data_ptr(), grad.data_ptr(), exp_avg.data_ptr(),
            exp_avg_sq.data_ptr(), _p(param_bf16), float(lr), float(beta1), float(beta2),
            float(eps), float(weight_decay), int(adamw), int(step), _p(grad_scale)]
    if zero_grad:
        _lib.call("mmpt_adam_step_zero_grad", *args, int(max_blocks), _stream())
    else:
        _lib.call("mmpt_adam_step", *args, _stream())


def clip_coef(sumsq, max_norm: float, coef) -> None:
    _lib.call("mmpt_clip_coef", sumsq.data_ptr(), float(max_norm), coef.data_ptr(), _stream())


def cast_f32_bf16(src, dst) -> None:
    _lib.call("mmpt_cast_f32_bf16", src.numel(), src.data_ptr(), dst.data_ptr(), _stream())


def transpose_bf16_batched(src_flat, dst_flat, desc, total_tiles: int) -> None:
    """Every weight's W^T in one launch: desc = device int64 [n, 4] {offset, rows, cols,
    first tile} into the flat bf16 buffers src_flat / dst_flat."""
    _check(desc, torch.int64, "transpose_batched.desc")
    _lib.call("mmpt_transpose_bf16_batched", desc.shape[0], desc.data_ptr(), int(total_tiles),
              src_flat.data_ptr(), dst_flat.data_ptr(), _stream())


def transpose_bf16(src, dst) -> None:
    rows, cols = src.shape
    if tuple(dst.shape) != (cols, rows):
        raise ValueError("transpose: dst must be [cols, rows]")
    _lib.call("mmpt_transpose_bf16", rows, cols, src.data_ptr(), _ld(src), dst.data_ptr(),
              _ld(dst), _stream())
