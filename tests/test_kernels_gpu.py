"""Op-level numerics of every HIP kernel in libmmpt.so against a plain PyTorch
fp32 reference of the same op (inputs rounded to bf16 where the kernel reads
bf16).  Calls go through the C-ABI (ctypes) — no ATen compute in the product
path.  Tolerances are written per test."""

import math

import pytest
import torch

pytestmark = pytest.mark.gpu

dev = "cuda"


@pytest.fixture(scope="module")
def K():
    from multimodal_llm_pretraining_amd import kernels

    return kernels


def bf(x):
    return x.to(torch.bfloat16)


def relerr(a, b):
    a = a.float()
    b = b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


# ------------------------------------------------------------------ GEMM
GEMM_SHAPES = [(256, 256, 256), (300, 136, 200), (97, 64, 64), (1000, 520, 776), (64, 8, 8)]


@pytest.mark.parametrize("M,N,Kd", GEMM_SHAPES)
@pytest.mark.parametrize("la,lb", [(0, 0), (0, 1), (1, 1), (1, 0)])
def test_gemm_layouts(K, M, N, Kd, la, lb):
    if (la == 1 and M % 8) or (lb == 1 and N % 8):
        pytest.skip("contiguous dim must be a multiple of 8")
    torch.manual_seed(0)
    A = bf(torch.randn(M, Kd, device=dev))
    B = bf(torch.randn(N, Kd, device=dev))
    a_st = A if la == 0 else A.t().contiguous()
    b_st = B if lb == 0 else B.t().contiguous()
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    K.gemm(a_st, b_st, out, layout_a=la, layout_b=lb)
    ref = A.float() @ B.float().t()
    assert relerr(out, ref) < 5e-3


def test_gemm_epilogues(K):
    torch.manual_seed(1)
    M, N, Kd = 333, 264, 320
    A = bf(torch.randn(M, Kd, device=dev))
    W = bf(torch.randn(N, Kd, device=dev) * 0.05)
    bias = bf(torch.randn(N, device=dev))
    acc = A.float() @ W.float().t()
    # bias
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    K.gemm(A, W, out, bias=bias)
    assert relerr(out, acc + bias.float()) < 5e-3
    # bias + GELU (pre and act)
    pre = torch.empty_like(out)
    act = torch.empty_like(out)
    K.gemm(A, W, pre, epilogue=K.EPI_BF16_GELU, bias=bias, out2=act)
    ref_pre = bf(acc + bias.float())
    assert relerr(pre, ref_pre) < 5e-3
    assert relerr(act, torch.nn.functional.gelu(ref_pre.float())) < 5e-3
    # dGELU
    dg = torch.empty_like(out)
    K.gemm(A, W, dg, epilogue=K.EPI_BF16_DGELU, aux=pre)
    x = pre.float().requires_grad_()
    torch.nn.functional.gelu(x).backward(bf(acc).float())
    assert relerr(dg, x.grad) < 5e-3
    # f32 store / accumulate
    c = torch.zeros(M, N, device=dev)
    K.gemm(A, W, c, epilogue=K.EPI_F32_STORE)
    assert relerr(c, acc) < 5e-3
    K.gemm(A, W, c, epilogue=K.EPI_F32_ACC)
    assert relerr(c, 2 * acc) < 5e-3
    # residual (+ aux)
    resid = torch.randn(M, N, device=dev)
    aux = bf(torch.randn(M, N, device=dev))
    o = torch.empty(M, N, device=dev)
    K.gemm(A, W, o, epilogue=K.EPI_F32_RESID, bias=bias, aux=aux, out2=resid)
    ref = resid + bf(bf(acc + bias.float()).float() + aux.float()).float()
    assert relerr(o, ref) < 5e-3


@pytest.mark.parametrize("M,N", [(333, 264), (4104, 4096)])
def test_gemm_quick_gelu_epilogues(K, M, N):
    """CLIP's quick-GELU epilogues against torch running the same ops on bf16 tensors ON
    THE CPU (the oracle's autocast: x*sigmoid(1.702x) as three bf16 ops, and autograd's
    bf16 backward through them).  Bit-exact on ≥ 99.9% of outputs, ≤ 1 bf16 ulp
    elsewhere (measured: bit-exact; torch's own ROCm kernels differ from the CPU on 14% of
    the backward outputs — scripts/diag/diag_qgelu.py — so the CPU is the reference)."""
    torch.manual_seed(5)
    Kd = 320
    A = bf(torch.randn(M, Kd, device=dev))
    W = bf(torch.randn(N, Kd, device=dev) * 0.1)
    bias = bf(torch.randn(N, device=dev))
    acc = A.float() @ W.float().t()
    pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    act = torch.empty_like(pre)
    K.gemm(A, W, pre, epilogue=K.EPI_BF16_QGELU, bias=bias, out2=act)
    assert relerr(pre, bf(acc + bias.float())) < 5e-3
    x = pre.cpu().requires_grad_()
    y = x * torch.sigmoid(1.702 * x)  # bf16 tensor ops, as under autocast
    assert y.dtype == torch.bfloat16

    def close(got, ref):
        d = (got.cpu().float() - ref.float()).abs()
        ulp = ref.float().abs().clamp_min(1e-30) * 2.0 ** -7
        return (d == 0).float().mean().item() >= 0.999 and bool((d <= ulp + 1e-30).all())

    assert close(act, y.detach())
    dg = torch.empty_like(pre)
    K.gemm(A, W, dg, epilogue=K.EPI_BF16_DQGELU, aux=pre)
    # the incoming gradient is the GEMM's own bf16(acc): take it from the plain epilogue
    # (same kernel, same accumulation order) rather than from torch's fp32 matmul
    gacc = torch.empty_like(pre)
    K.gemm(A, W, gacc)
    y.backward(gacc.cpu())
    assert close(dg, x.grad)
    # the fused bias-gradient column sums
    db = torch.zeros(N, device=dev)
    dg2 = torch.empty_like(pre)
    K.gemm_dgelu_colsum(A, W, dg2, pre, db, quick=True)
    assert torch.equal(dg2, dg)
    assert relerr(db, dg.float().sum(0).to(torch.bfloat16).float()) < 2e-3  # bf16 grad_bias


def test_layernorm_f32(K):
    """fp32-output LayerNorm (CLIP pre_layrnorm) fwd/bwd vs torch fp32."""
    torch.manual_seed(6)
    rows, h, eps = 577 * 3, 1024, 1e-5
    x = torch.randn(rows, h, device=dev) * 2 + 0.5
    w = torch.randn(h, device=dev)
    b = torch.randn(h, device=dev)
    y = torch.empty(rows, h, device=dev)
    mean, rstd = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
    K.layernorm_f32_fwd(x, w, b, eps, y, mean, rstd)
    xr, wr, br = (t.clone().requires_grad_() for t in (x, w, b))
    ref = torch.nn.functional.layer_norm(xr, (h,), wr, br, eps)
    assert relerr(y, ref) < 1e-6
    dy = torch.randn(rows, h, device=dev)
    ref.backward(dy)
    dx = torch.empty_like(x)
    dw, db = torch.ones(h, device=dev), torch.zeros(h, device=dev)
    K.layernorm_f32_bwd(x, mean, rstd, dy, w, dx, dw, db)
    assert relerr(dx, xr.grad) < 1e-5
    assert relerr(dw - 1, wr.grad) < 1e-5 and relerr(db, br.grad) < 1e-5


@pytest.mark.parametrize("patch,image", [(14, 56), (16, 64)])
def test_im2col_padded(K, patch, image):
    torch.manual_seed(7)
    B, C = 3, 3
    pix = torch.rand(B, C, image, image, device=dev)
    kk = C * patch * patch
    kp = (kk + 7) // 8 * 8
    G = image // patch
    cols = torch.full((B * G * G, kp), 7.0, device=dev, dtype=torch.bfloat16)
    K.im2col(pix, patch, cols)
    ref = pix.unfold(2, patch, patch).unfold(3, patch, patch)  # B C G G p p
    ref = ref.permute(0, 2, 3, 1, 4, 5).reshape(B * G * G, kk)
    assert torch.equal(cols[:, :kk], bf(ref))
    assert torch.all(cols[:, kk:] == 0)


@pytest.mark.parametrize("la,lb", [(0, 0), (0, 1), (1, 1)])
def test_gemm_big_tile(K, la, lb):
    """M, N large enough for the 256x256 / 8-wave tile, ragged M and K tails."""
    torch.manual_seed(11)
    M, N, Kd = 4104 if la == 0 else 4096, 4096, 200
    A = bf(torch.randn(M, Kd, device=dev))
    B = bf(torch.randn(N, Kd, device=dev))
    a_st = A if la == 0 else A.t().contiguous()
    b_st = B if lb == 0 else B.t().contiguous()
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    K.gemm(a_st, b_st, out, layout_a=la, layout_b=lb)
    assert relerr(out, A.float() @ B.float().t()) < 5e-3


@pytest.mark.parametrize("Kd", [8, 72, 200, 2048, 4160])
@pytest.mark.parametrize("la,lb", [(0, 0), (1, 1), (0, 1), (1, 0)])
def test_gemm_bigtile_pipeline_elementwise(K, Kd, la, lb):
    """The big-tile path (gemm4p; mixed layouts: gemm128): every output element (not a norm) against fp32, for
    K-tile counts 1, 2, 4 (tails), 32 and 65 (the steady-state DMA ring), ragged M/N.
    fp32 output (F32_STORE rounds to bf16 once): |err| <= 2^-8 |ref| + fp32 order noise."""
    from multimodal_llm_pretraining_amd import _lib
    import ctypes

    M, N = (4104, 4100) if la == 0 and lb == 0 else (4096, 4104)
    tile, splits = ctypes.c_int(0), ctypes.c_int(0)
    _lib.call("mmpt_gemm_plan", M, N, Kd, K.EPI_F32_STORE, 0, ctypes.byref(tile), ctypes.byref(splits))
    assert tile.value == 256 and splits.value == 1
    torch.manual_seed(100 + Kd)
    A = bf(torch.randn(M, Kd, device=dev))
    B = bf(torch.randn(N, Kd, device=dev))
    a_st = A if la == 0 else A.t().contiguous()
    b_st = B if lb == 0 else B.t().contiguous()
    out = torch.full((M, N), float("nan"), device=dev)
    K.gemm(a_st, b_st, out, layout_a=la, layout_b=lb, epilogue=K.EPI_F32_STORE)
    ref = A.float() @ B.float().t()
    err = (out - ref).abs()
    tol = 4e-3 * ref.abs() + 1e-5 * Kd
    bad = (~(err <= tol)).sum().item()
    assert bad == 0, f"{bad} elements off; max err {err.max().item()}"


@pytest.mark.parametrize("Kd,M,N", [(18464, 4096, 4096), (34784, 2560, 10240), (1000, 8192, 8192)])
def test_gemm4p_k_tail_weight_gradient(K, Kd, M, N):
    """Round 5: weight gradients whose K (the token count) is not a multiple of 64 run gemm4p's
    K-tail form (the last K-tile's pieces past K read zeros from an out-of-range buffer offset),
    split-K included — C5's tower / LLM at micro-batch 32 (18464 = 32 x 577, 34784 = 32 x 1087).
    F32_ACC into a non-zero gradient: every element against fp32 (bf16-rounded product + old)."""
    torch.manual_seed(Kd)
    dY = bf(torch.randn(Kd, M, device=dev))  # K_ROWS: [tokens][out features]
    X = bf(torch.randn(Kd, N, device=dev))
    G0 = torch.randn(M, N, device=dev)
    G = G0.clone()
    K.gemm(dY, X, G, layout_a=K.K_ROWS, layout_b=K.K_ROWS, epilogue=K.EPI_F32_ACC)
    assert K.gemm_last_kernel().startswith("gemm4p_kt_kernel"), K.gemm_last_kernel()
    prod = dY.float().t() @ X.float()
    ref = G0 + prod.to(torch.bfloat16).float()
    err = (G - ref).abs()
    tol = 2.0 ** -7 * prod.abs() + 1e-5 * Kd ** 0.5 + 1e-6 * G0.abs()
    bad = (~(err <= tol)).sum().item()
    assert bad == 0, f"{bad} elements off; max err {err.max().item()}"


@pytest.mark.parametrize("epi", ["bf16", "gelu", "dgelu", "acc", "resid"])
def test_gemm_bigtile_epilogues(K, epi):
    """Fused epilogues on the big-tile kernel (M, N ragged)."""
    torch.manual_seed(7)
    M, N, Kd = 4104, 4100, 264
    A = bf(torch.randn(M, Kd, device=dev))
    W = bf(torch.randn(N, Kd, device=dev) * 0.05)
    bias = bf(torch.randn(N, device=dev))
    acc = A.float() @ W.float().t()
    if epi == "bf16":
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        K.gemm(A, W, out, bias=bias)
        assert relerr(out, acc + bias.float()) < 5e-3
    elif epi == "gelu":
        pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        act = torch.empty_like(pre)
        K.gemm(A, W, pre, epilogue=K.EPI_BF16_GELU, bias=bias, out2=act)
        ref_pre = bf(acc + bias.float())
        assert relerr(pre, ref_pre) < 5e-3
        assert relerr(act, torch.nn.functional.gelu(ref_pre.float())) < 5e-3
    elif epi == "dgelu":
        pre = bf(torch.randn(M, N, device=dev))
        dg = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        K.gemm(A, W, dg, epilogue=K.EPI_BF16_DGELU, aux=pre)
        x = pre.float().requires_grad_()
        torch.nn.functional.gelu(x).backward(bf(acc).float())
        assert relerr(dg, x.grad) < 5e-3
    elif epi == "acc":
        c = torch.ones(M, N, device=dev)
        K.gemm(A, W, c, epilogue=K.EPI_F32_ACC)
        assert relerr(c - 1, acc) < 5e-3
    else:
        resid = torch.randn(M, N, device=dev)
        aux = bf(torch.randn(M, N, device=dev))
        o = torch.empty(M, N, device=dev)
        K.gemm(A, W, o, epilogue=K.EPI_F32_RESID, bias=bias, aux=aux, out2=resid)
        ref = resid + bf(bf(acc + bias.float()).float() + aux.float()).float()
        assert relerr(o, ref) < 5e-3


@pytest.mark.parametrize("epi", ["bf16", "gelu"])
@pytest.mark.parametrize("Kd", [256, 2048])
def test_gemm_bigtile_persistent_vs_one_round_bitwise(K, epi, Kd):
    """A persistent launch with several tiles per workgroup (the next tile's DMA in flight under
    each epilogue, counted waits that leave the epilogue's stores in flight) against one tile
    per workgroup (a 4096-row slice: 256 tiles).  Same per-element arithmetic, so the two must
    agree bitwise — a wrong wait count or a tile stored from the wrong accumulators shows here."""
    torch.manual_seed(31 + Kd)
    M, N = 16384, 4096
    A = bf(torch.randn(M, Kd, device=dev))
    W = bf(torch.randn(N, Kd, device=dev) * 0.05)
    bias = bf(torch.randn(N, device=dev))
    gelu = epi == "gelu"
    kw = dict(epilogue=K.EPI_BF16_GELU) if gelu else {}
    full = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    full2 = torch.empty_like(full) if gelu else None
    K.gemm(A, W, full, bias=bias, out2=full2, **kw)
    sl = torch.empty(4096, N, device=dev, dtype=torch.bfloat16)
    sl2 = torch.empty_like(sl) if gelu else None
    for r in range(0, M, 4096):
        K.gemm(A[r:r + 4096], W, sl, bias=bias, out2=sl2, **kw)
        assert torch.equal(full[r:r + 4096], sl), f"rows {r}.. differ"
        if gelu:
            assert torch.equal(full2[r:r + 4096], sl2), f"GELU rows {r}.. differ"


@pytest.mark.parametrize("M,N,Kd", [(4104, 4100, 264), (333, 264, 320), (45248 // 8, 8192, 2048)])
def test_gemm_dgelu_colsum(K, M, N, Kd):
    """EPI_BF16_DGELU_COLSUM: the dGELU output bitwise as EPI_BF16_DGELU, and the fused
    bias gradient == bf16(Σ_rows of that bf16 output) accumulated into fp32."""
    torch.manual_seed(21)
    A = bf(torch.randn(M, Kd, device=dev))
    W = bf(torch.randn(N, Kd, device=dev) * 0.05)
    pre = bf(torch.randn(M, N, device=dev))
    ref = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    K.gemm(A, W, ref, epilogue=K.EPI_BF16_DGELU, aux=pre)
    out = torch.empty_like(ref)
    db = torch.full((N,), 0.5, device=dev)
    K.gemm_dgelu_colsum(A, W, out, pre, db)
    assert torch.equal(out, ref)
    want = ref.float().sum(0).to(torch.bfloat16).float() + 0.5
    assert relerr(db, want) < 2e-3


@pytest.mark.parametrize("M,N,Kd", [(20232, 4096, 256), (4104, 6144, 2048), (333, 512, 320)])
def test_gemm_bigtile_staged_stores_every_element(K, M, N, Kd):
    """The LDS-staged epilogue stores (whole-width tiles, several tiles per persistent
    workgroup, ragged M): the bf16 output must equal the F32_STORE output (= f32(bf16(acc)),
    per-lane stores) bit for bit, and GELU's two outputs must be consistent element by
    element — a row or column staged to the wrong place, or a slot overwritten by the next
    tile's prologue DMA, shows here."""
    torch.manual_seed(41 + Kd)
    A = bf(torch.randn(M, Kd, device=dev))
    W = bf(torch.randn(N, Kd, device=dev) * 0.05)
    o16 = torch.full((M, N), float("nan"), device=dev).to(torch.bfloat16)
    K.gemm(A, W, o16)
    o32 = torch.full((M, N), float("nan"), device=dev)
    K.gemm(A, W, o32, epilogue=K.EPI_F32_STORE)
    assert torch.equal(o16.float(), o32)
    bias = bf(torch.randn(N, device=dev))
    pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    act = torch.empty_like(pre)
    K.gemm(A, W, pre, epilogue=K.EPI_BF16_GELU, bias=bias, out2=act)
    ref_pre = bf(A.float() @ W.float().t() + bias.float())
    assert relerr(pre, ref_pre) < 5e-3
    # fp64 erfc form (torch's fp32 GELU cancels in 1 + erf(x/sqrt 2) for x < -4)
    x64 = pre.double()
    want = (0.5 * x64 * torch.special.erfc(-x64 / 2 ** 0.5)).to(torch.bfloat16)
    assert torch.equal(act, want)
    dg = torch.empty_like(pre)
    K.gemm(A, W, dg, epilogue=K.EPI_BF16_DGELU, aux=pre)
    x = pre.float().requires_grad_()
    torch.nn.functional.gelu(x).backward(o16.float())
    assert relerr(dg, x.grad) < 5e-3


@pytest.mark.parametrize("inplace", [False, True])
@pytest.mark.parametrize("M,N,Kd", [(20232, 2048, 256), (4104, 4096, 1024)])
def test_gemm_bigtile_residual_bitwise(K, M, N, Kd, inplace):
    """The residual epilogue (fc2 / attention-dense forward, pipelined whole-width rows):
    without a bias, C = C2 + bf16(f32(bf16(acc)) + aux) exactly, with f32(bf16(acc)) taken from
    the F32_STORE epilogue of the same GEMM — bitwise on every element, C2 aliasing C (the
    residual stream updated in place, as the model does) or not."""
    torch.manual_seed(51 + Kd)
    A = bf(torch.randn(M, Kd, device=dev))
    W = bf(torch.randn(N, Kd, device=dev) * 0.05)
    accb = torch.empty(M, N, device=dev)
    K.gemm(A, W, accb, epilogue=K.EPI_F32_STORE)
    aux = bf(torch.randn(M, N, device=dev))
    resid = torch.randn(M, N, device=dev)
    want = resid + bf(accb + aux.float()).float()
    if inplace:
        out = resid.clone()
        K.gemm(A, W, out, epilogue=K.EPI_F32_RESID, aux=aux, out2=out)
    else:
        out = torch.full((M, N), float("nan"), device=dev)
        K.gemm(A, W, out, epilogue=K.EPI_F32_RESID, aux=aux, out2=resid)
    assert torch.equal(out, want)


def test_gemm_bigtile_deterministic_under_repeat(K):
    """Same inputs, 5 launches: bitwise identical (an LDS race shows up as flicker)."""
    torch.manual_seed(3)
    M, N, Kd = 8192, 4096, 2048
    A = bf(torch.randn(M, Kd, device=dev))
    B = bf(torch.randn(N, Kd, device=dev))
    outs = []
    for _ in range(5):
        o = torch.empty(M, N, device=dev)
        K.gemm(A, B, o, epilogue=K.EPI_F32_STORE)
        outs.append(o)
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    ref = A.float() @ B.float().t()
    assert ((outs[0] - ref).abs() <= 4e-3 * ref.abs() + 1e-2).all()


@pytest.mark.parametrize("M,N,Kd", [(256, 256, 8200), (2048, 768, 12608), (6144, 2048, 45248)])
def test_gemm_splitk_weight_grad(K, M, N, Kd):
    """dW = dY^T X with K = tokens: split-K slabs + ordered reduce == single pass."""
    from multimodal_llm_pretraining_amd import _lib

    assert _lib.query("mmpt_gemm_workspace_bytes", M, N, Kd, K.EPI_F32_ACC) > 0
    torch.manual_seed(12)
    dY = bf(torch.randn(Kd, M, device=dev))
    X = bf(torch.randn(Kd, N, device=dev))
    G = torch.ones(M, N, device=dev)
    K.gemm(dY, X, G, layout_a=K.K_ROWS, layout_b=K.K_ROWS, epilogue=K.EPI_F32_ACC)
    ref = dY.float().t() @ X.float()
    assert relerr(G - 1, ref) < 5e-3
    G2 = torch.empty(M, N, device=dev)
    K.gemm(dY, X, G2, layout_a=K.K_ROWS, layout_b=K.K_ROWS, epilogue=K.EPI_F32_STORE)
    assert relerr(G2, ref) < 5e-3
    G3 = torch.empty(M, N, device=dev)
    K.gemm(dY, X, G3, layout_a=K.K_ROWS, layout_b=K.K_ROWS, epilogue=K.EPI_F32_STORE)
    assert torch.equal(G2, G3)  # deterministic


def _bf16_ulp(x: torch.Tensor) -> torch.Tensor:
    """Spacing of bf16 at |x| (the bias gradient is rounded to bf16 once)."""
    e = torch.floor(torch.log2(x.abs().clamp_min(1e-30)))
    return torch.pow(2.0, e - 7)


@pytest.mark.parametrize("M,N,Kd,form", [(6144, 2048, 45248, "split"), (2048, 8192, 180992, "acc"),
                                         (2296, 776, 50432, "split"), (4000, 4000, 8192, "acc"),
                                         (2304, 768, 50432, "split"),
                                         # round 6: K % 64 != 0 (32 samples x 707 tokens), K-tail form
                                         (6144, 2048, 22624, "split"), (2048, 8192, 22624, "acc"),
                                         (2048, 2048, 22600, "split")])
def test_gemm_wgrad_colsum(K, M, N, Kd, form):
    """Round 5: weight + bias gradient in one pass (EPI_F32_ACC_COLSUM): the weight gradient is
    bitwise the plain F32_ACC one (same plan, same MFMA order), and the bias gradient — the dY
    fragments the MFMAs read, summed per K split, reduced in fixed order — is bf16(Σ_rows dY)
    within one bf16 unit of fp64 (the separate column-sum pass is held to the same bar).
    The fp32 sums' own rounding is allowed a floor of 4 x 2^-24 x Σ|dY| (near-zero sums).
    Shapes: Pythia qkv (K cut to a quarter) / fc2 (full K, no split), ragged M and N (split and
    not), ViT qkv."""
    from multimodal_llm_pretraining_amd import _lib

    rows = _lib.query("mmpt_gemm_acc_colsum_rows", M, N, Kd)
    tn = (N + 255) // 256
    assert rows % tn == 0 and (rows > tn) == (form == "split"), rows
    torch.manual_seed(M + Kd)
    dY = bf(torch.randn(Kd, M, device=dev) * 1e-2)
    X = bf(torch.randn(Kd, N, device=dev))
    G0 = torch.randn(M, N, device=dev)
    db0 = torch.randn(M, device=dev)
    G, db, db2 = G0.clone(), db0.clone(), torch.zeros(M, device=dev)
    assert K.gemm_wgrad_colsum(dY, X, G, db, db2)
    name = K.gemm_last_kernel()
    kern = "gemm4p_kernel" if Kd % 64 == 0 else "gemm4p_kt_kernel"
    assert name == f"{kern}<1, 1, {102 if form == 'split' else 12}>", name
    Gr = G0.clone()
    K.gemm(dY, X, Gr, layout_a=K.K_ROWS, layout_b=K.K_ROWS, epilogue=K.EPI_F32_ACC)
    assert torch.equal(G, Gr), "weight gradient differs from the plain F32_ACC pass"
    ref = dY.double().sum(0)
    tol = _bf16_ulp(ref.float()).double() + 4 * 2.0 ** -24 * dY.double().abs().sum(0)
    fused = db - db0
    assert ((fused.double() - ref).abs() <= tol).all(), \
        (fused.double() - ref).abs().div(tol).max().item()
    assert ((db2.double() - ref).abs() <= tol).all()  # the second bias (dbias2)
    sep = torch.zeros(M, device=dev)
    K.colsum(dY, sep, accumulate=True)
    assert ((sep.double() - ref).abs() <= tol).all()
    # deterministic: a second fused pass gives the same bits
    G2, dbb = G0.clone(), db0.clone()
    K.gemm_wgrad_colsum(dY, X, G2, dbb)
    assert torch.equal(G2, G) and torch.equal(dbb, db)


def test_gemm_wgrad_colsum_without_workspace(K):
    """F32_ACC_COLSUM called without a workspace runs one K split: it writes that split's
    partial rows (one per 256-column tile) and zeroes the other planned rows, so the fixed-order reduce over mmpt_gemm_acc_colsum_rows
    rows still gives the bias gradient (C-ABI level: the Python wrapper always passes one)."""
    from multimodal_llm_pretraining_amd import _lib

    M, N, Kd = 2048, 2048, 45248
    rows = _lib.query("mmpt_gemm_acc_colsum_rows", M, N, Kd)
    assert rows > 8
    torch.manual_seed(3)
    dY = bf(torch.randn(Kd, M, device=dev))
    X = bf(torch.randn(Kd, N, device=dev))
    G = torch.zeros(M, N, device=dev)
    part = torch.full((rows, M), float("nan"), device=dev)
    st = torch.cuda.current_stream().cuda_stream
    _lib.call("mmpt_gemm_bf16", K.K_ROWS, K.K_ROWS, K.EPI_F32_ACC_COLSUM, M, N, Kd,
              dY.data_ptr(), M, X.data_ptr(), N, G.data_ptr(), N, None, None, 0,
              part.data_ptr(), M, None, 0, st)
    assert K.gemm_last_kernel() == "gemm4p_kernel<1, 1, 12>"
    assert (part[8:] == 0).all()  # one split: 8 column tiles written, the rest zeroed
    assert not torch.isnan(part).any()
    db = torch.zeros(M, device=dev)
    _lib.call("mmpt_colsum_f32", rows, M, part.data_ptr(), db.data_ptr(), None, 1, st)
    ref = dY.double().sum(0)
    tol = _bf16_ulp(ref.float()).double() + 4 * 2.0 ** -24 * dY.double().abs().sum(0)
    assert ((db.double() - ref).abs() <= tol).all()
    # shapes the fused form does not take: the query says 0 and the wrapper declines
    assert _lib.query("mmpt_gemm_acc_colsum_rows", 768, 768, 50432) == 0
    assert _lib.query("mmpt_gemm_acc_colsum_rows", 2048, 2048, 22600) > 0  # K-tail form (r6)
    small = bf(torch.randn(640, 768, device=dev))
    assert not K.gemm_wgrad_colsum(small, bf(torch.randn(640, 768, device=dev)),
                                   torch.zeros(768, 768, device=dev), torch.zeros(768, device=dev))


def test_gemm_wgrad_colsum_ignores_krev(K):
    """the fused bias-gradient row sums split a tile row's K-tiles between its
    columns by loop index, so a reversed K walk on some columns would sum some K-tiles twice
    and others not at all.  With MMPT_GEMM_KREV=1 the fused form still walks K forward: bitwise
    the KREV=0 results (weight and bias gradient), at a shape with more tiles than CUs."""
    from multimodal_llm_pretraining_amd import _lib

    M, N, Kd = 2048, 256 * 40, 8192  # 320 tiles > 256 workgroups: second tiles exist
    torch.manual_seed(31)
    dY = bf(torch.randn(Kd, M, device=dev) * 1e-2)
    X = bf(torch.randn(Kd, N, device=dev))

    def run():
        G, db = torch.zeros(M, N, device=dev), torch.zeros(M, device=dev)
        assert K.gemm_wgrad_colsum(dY, X, G, db)
        return G, db

    prev = _lib.set_switch("MMPT_GEMM_KREV", 0)
    try:
        g0, b0 = run()
        _lib.set_switch("MMPT_GEMM_KREV", 1)
        g1, b1 = run()
    finally:
        _lib.set_switch("MMPT_GEMM_KREV", prev)
    assert torch.equal(g0, g1) and torch.equal(b0, b1)
    ref = dY.double().sum(0)
    tol = _bf16_ulp(ref.float()).double() + 4 * 2.0 ** -24 * dY.double().abs().sum(0)
    assert ((b1.double() - ref).abs() <= tol).all()


@pytest.mark.parametrize("la,epi,M,N,Kd", [(0, "bf16", 256 * 41, 2048, 1024),
                                             (0, "resid", 256 * 41, 2048, 1024),
                                             (1, "f32", 2048, 256 * 40, 256 * 41)])
def test_gemm4p_reversed_k_walk(K, la, epi, M, N, Kd):
    """MMPT_GEMM_KREV: a persistent workgroup's odd tiles walk K last-to-first (the A K-slices
    the previous tile round loaded last are read first, from L2).  More tiles than CUs, so
    workgroups run a second (reversed) tile; every element against the fp32 product, and the
    forward-order results within the rounding of a different fp32 summation order."""
    from multimodal_llm_pretraining_amd import _lib

    torch.manual_seed(21)
    if la == 0:
        A, W = bf(torch.randn(M, Kd, device=dev)), bf(torch.randn(N, Kd, device=dev))
        acc = A.float() @ W.float().t()
    else:  # weight-gradient form (K_ROWS x K_ROWS), split-K planned by the library
        A, W = bf(torch.randn(Kd, M, device=dev)), bf(torch.randn(Kd, N, device=dev))
        acc = A.float().t() @ W.float()

    def run():
        if la == 1:
            c = torch.zeros(M, N, device=dev)
            K.gemm(A, W, c, layout_a=1, layout_b=1, epilogue=K.EPI_F32_STORE)
            return c
        if epi == "resid":
            c = torch.randn(M, N, device=dev, generator=torch.Generator(device=dev).manual_seed(2))
            K.gemm(A, W, c, epilogue=K.EPI_F32_RESID, out2=c)
            return c
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        K.gemm(A, W, c)
        return c

    # (the weight-gradient form as the all-split launch: the tail split runs its 320 tiles as
    # one unsplit round of 240 + a split tail, one tile per workgroup, so nothing walks reversed)
    prev = _lib.set_switch("MMPT_GEMM_KREV", 0)
    prev_w = _lib.set_switch("MMPT_GEMM_WTAIL", 0)
    try:
        fwd = run()
        _lib.set_switch("MMPT_GEMM_KREV", 1)
        rev = run()
    finally:
        _lib.set_switch("MMPT_GEMM_KREV", prev)
        _lib.set_switch("MMPT_GEMM_WTAIL", prev_w)
    base = 0.0
    if epi == "resid":
        base = torch.randn(M, N, device=dev, generator=torch.Generator(device=dev).manual_seed(2))
        acc = acc + base
    assert relerr(rev, acc) < 5e-3
    # every epilogue here rounds the product to bf16 first (plain output, the residual's branch,
    # F32_STORE = f32(bf16(acc))): a different fp32 summation order may land on a neighbouring
    # bf16 value
    prod = (acc - base).abs()
    tol = 2.0 ** -7
    d = (rev.float() - fwd.float()).abs()
    assert bool((d <= tol * prod + 1e-5 * fwd.float().abs() + 1e-4 * prod.max()).all())
    assert not torch.equal(rev, fwd)  # the reversed walk did run (a different summation order)


@pytest.mark.parametrize("M,epi", [(256 * 35, "bf16"), (256 * 34 + 100, "bf16"),
                                   (256 * 35, "resid"), (256 * 34 + 100, "resid"),
                                   (256 * 32 + 16, "bf16"), (256 * 32 + 16, "resid"),
                                   (256 * 32 + 100, "resid")])
def test_gemm_tail_split(K, M, epi):
    """The tail split (MMPT_GEMM_TAIL): the bottom tile rows that would run as a partial last
    round (35 tile rows x 8 = 280 tiles = 1 round + 24) run as a split-K GEMM + epilogue
    kernel.  Rows above the tail are bitwise the single-launch result; the tail rows are the
    same epilogue formula on a differently ordered fp32 sum (within one bf16 rounding of it)
    and match the fp32 product; bias, the residual's aux branch and a partial last tile.
    Tails of <= 128 rows (16 = C2's 16 x 2049 tokens) run on the 128-row kernel."""
    from multimodal_llm_pretraining_amd import _lib

    torch.manual_seed(22)
    N, Kd = 2048, 2048
    A, W = bf(torch.randn(M, Kd, device=dev)), bf(torch.randn(N, Kd, device=dev))
    bias = bf(torch.randn(N, device=dev))
    aux = bf(torch.randn(M, N, device=dev))
    acc = A.float() @ W.float().t()
    res0 = torch.randn(M, N, device=dev)

    def run():
        if epi == "resid":
            c = res0.clone()
            K.gemm(A, W, c, epilogue=K.EPI_F32_RESID, bias=bias, aux=aux, out2=c)
        else:
            c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            K.gemm(A, W, c, bias=bias)
        return c, _lib.query("mmpt_gemm_last_tail_rows")

    prev = _lib.set_switch("MMPT_GEMM_TAIL", 0)
    try:
        ref, t0 = run()
        _lib.set_switch("MMPT_GEMM_TAIL", 1)
        got, mt = run()
    finally:
        _lib.set_switch("MMPT_GEMM_TAIL", prev)
    assert t0 == 0 and mt == M - 32 * 256
    m0 = M - mt
    assert torch.equal(got[:m0], ref[:m0])
    want = acc + bias.float()
    if epi == "resid":
        want = res0 + bf(bf(acc + bias.float()).float() + aux.float()).float()
    assert relerr(got[m0:], want[m0:]) < 5e-3
    # one bf16 rounding of (acc + bias) may land on the neighbouring value; the residual form
    # rounds again after adding aux: |d| <= ulp(acc + bias) + ulp(v + aux) <= 2^-7 (2|acc + bias|
    # + |aux|), the fp32 residual add ~1e-7 relative; and the two fp32 sums themselves differ by
    # their rounding (K = 2048 products of N(0,1) values: ~1e-4, bounded here by 2e-3)
    prod = (acc + bias.float()).abs()[m0:]
    d = (got[m0:].float() - ref[m0:].float()).abs()
    lim = 2.0 ** -7 * (2 * prod + (aux.float().abs()[m0:] if epi == "resid" else 0))
    assert bool((d <= lim + 1e-6 * ref[m0:].float().abs() + 2e-3).all())


@pytest.mark.parametrize("M,N,Kd,epi,mode", [(5120, 3328, 8192, "acc", 1), (5120, 3328, 8208, "acc", 1),
                                             (5120, 3328, 8192, "store", 1),
                                             (3328, 5120, 8192, "acc", 2), (3328, 5120, 8208, "store", 2),
                                             (5120, 3328, 8192, "colsum", 1), (5120, 3328, 8208, "colsum", 1),
                                             (3328, 5120, 8192, "colsum", 2)])
def test_gemm_wgrad_tail_split(K, M, N, Kd, epi, mode):
    """The weight-gradient tail split (MMPT_GEMM_WTAIL, round 6): a split-K weight gradient whose
    tiles make a partial round runs its whole rounds' tile rows (mode 1) or columns (mode 2,
    forced) unsplit straight into C and splits only the rest — against the all-split launch and
    the fp32 product: each output is bf16(sum) (+ C), the two sums differ only in fp32 order, so
    by at most one bf16 rounding of the product; K tails (8208) through the K-tail kernel."""
    from multimodal_llm_pretraining_amd import _lib

    torch.manual_seed(23)
    a, b = bf(torch.randn(Kd, M, device=dev)), bf(torch.randn(Kd, N, device=dev))
    c0 = torch.randn(M, N, device=dev)
    e = K.EPI_F32_STORE if epi == "store" else K.EPI_F32_ACC
    db0 = torch.randn(M, device=dev)

    def run():
        c, db = c0.clone(), db0.clone()
        if epi == "colsum":  # + the fused bias-gradient row sums (dbias += bf16(sum_k a[k, m]))
            assert K.gemm_wgrad_colsum(a, b, c, db)
        else:
            K.gemm(a, b, c, layout_a=K.K_ROWS, layout_b=K.K_ROWS, epilogue=e)
        torch.cuda.synchronize()
        return c, K.gemm_last_kernel(), db

    prev = _lib.set_switch("MMPT_GEMM_WTAIL", 0)
    try:
        ref, k0, db_ref = run()
        _lib.set_switch("MMPT_GEMM_WTAIL", mode)
        got, k1, db_got = run()
    finally:
        _lib.set_switch("MMPT_GEMM_WTAIL", prev)
    # split (EPI_SPLIT 100 / EPI_SPLIT_CS 102) vs the unsplit main launch
    assert k0.endswith((", 100>", ", 102>")) and not k1.endswith((", 100>", ", 102>")), (k0, k1)
    if epi == "colsum":
        rs = a.double().sum(0)
        lim_b = 2.0 ** -7 * rs.abs() + 1e-3
        for dbv in (db_got, db_ref):
            assert bool(((dbv.double() - db0.double() - rs).abs() <= lim_b).all())
    prod = a.float().t() @ b.float()
    want = bf(prod).float() + (0 if epi == "store" else c0)
    lim = 2.0 ** -7 * prod.abs() + 1e-5 * want.abs() + 1e-3  # one bf16 step (up to 2^-7 relative)
    for out in (got, ref):
        assert bool(((out - want).abs() <= lim).all())
    assert bool(((got - ref).abs() <= 2 * lim).all())


@pytest.mark.parametrize("big", ["a", "b"])
def test_gemm_operand_over_2gib(K, big):
    """A ROWS_K operand past 2 GiB (fc2 forward / fc1 dX read 180,992 x 8192 bf16 = 2.97 GB at the
    bench micro-batch, lm_head dX 13 GB of dlogits): the LDS-DMA offsets are relative to the
    tile's first row, so rows past 2^31 bytes are read — an absolute offset would exceed the
    buffer resource's range and come back as zeros."""
    torch.manual_seed(3)
    Kd, R, S = 8192, 139264, 256  # 139,264 x 8192 x 2 B = 2.28 GB
    big_op = bf(torch.randn(R, Kd, device=dev))
    small = bf(torch.randn(S, Kd, device=dev))
    rows = torch.cat([torch.arange(0, 64), torch.arange(R - 9000, R, 37)]).to(dev)
    if big == "a":
        out = torch.empty(R, S, device=dev, dtype=torch.bfloat16)
        K.gemm(big_op, small, out)
        got, ref = out[rows].float(), big_op[rows].float() @ small.float().T
    else:
        out = torch.empty(S, R, device=dev, dtype=torch.bfloat16)
        K.gemm(small, big_op, out)
        got, ref = out[:, rows].float(), small.float() @ big_op[rows].float().T
    assert relerr(got, ref) < 1e-2


def test_gemm_rejects_bad_args(K):
    A = bf(torch.randn(64, 12, device=dev))
    with pytest.raises(RuntimeError):
        K.gemm(A, A, torch.empty(64, 64, device=dev, dtype=torch.bfloat16))


# ------------------------------------------------------------------ LayerNorm
@pytest.mark.parametrize("rows,h,eps", [(129, 2048, 1e-5), (77, 768, 1e-12), (5, 64, 1e-5)])
def test_layernorm_dual(K, rows, h, eps):
    torch.manual_seed(2)
    x = torch.randn(rows, h, device=dev) * 2 + 0.5
    w1, b1 = torch.randn(h, device=dev), torch.randn(h, device=dev)
    w2, b2 = torch.randn(h, device=dev), torch.randn(h, device=dev)
    y1 = torch.empty(rows, h, device=dev, dtype=torch.bfloat16)
    y2 = torch.empty_like(y1)
    mean = torch.empty(rows, device=dev)
    rstd = torch.empty(rows, device=dev)
    K.layernorm_fwd(x, w1, b1, eps, y1, mean, rstd, w2, b2, y2)
    xr = x.clone().requires_grad_()
    w1r, b1r, w2r, b2r = (t.clone().requires_grad_() for t in (w1, b1, w2, b2))
    r1 = torch.nn.functional.layer_norm(xr, (h,), w1r, b1r, eps)
    r2 = torch.nn.functional.layer_norm(xr, (h,), w2r, b2r, eps)
    assert relerr(y1, r1) < 4e-3 and relerr(y2, r2) < 4e-3
    dy1 = bf(torch.randn(rows, h, device=dev))
    dy2 = bf(torch.randn(rows, h, device=dev))
    dres = torch.randn(rows, h, device=dev)
    (r1 * dy1.float()).sum().add_((r2 * dy2.float()).sum()).backward()
    dx = torch.empty(rows, h, device=dev)
    dw1, db1, dw2, db2 = (torch.zeros(h, device=dev) for _ in range(4))
    K.layernorm_bwd(x, mean, rstd, dy1, w1, dx, dw1, db1, dy2, w2, dw2, db2, dresid=dres)
    assert relerr(dx, xr.grad + dres) < 1e-4
    for a, r in ((dw1, w1r), (db1, b1r), (dw2, w2r), (db2, b2r)):
        assert relerr(a, r.grad) < 1e-4
    # fused outputs: bf16 copy of dx and the bias gradient Σ_rows bf16(dx) (rounded to
    # bf16, accumulated into two fp32 targets); the single-LN form (ViT) too
    dxb = torch.empty(rows, h, device=dev, dtype=torch.bfloat16)
    ds1, ds2 = torch.ones(h, device=dev), torch.zeros(h, device=dev)
    dx2 = torch.empty(rows, h, device=dev)
    dw1b, db1b = torch.zeros(h, device=dev), torch.zeros(h, device=dev)
    K.layernorm_bwd(x, mean, rstd, dy1, w1, dx2, dw1b, db1b, dresid=dres, dx_bf16=dxb,
                    dsum=ds1, dsum2=ds2)
    assert torch.equal(dxb, dx2.to(torch.bfloat16))
    ref_sum = dxb.float().sum(0).to(torch.bfloat16).float()
    assert relerr(ds2, ref_sum) < 1e-5 and relerr(ds1 - 1, ref_sum) < 1e-5
    assert relerr(db1b, dy1.float().sum(0)) < 1e-4


@pytest.mark.parametrize("rows,h,dual", [(9001, 2048, True), (5003, 768, False), (4100, 64, True)])
def test_layernorm_fwd_persistent_bitwise(K, rows, h, dual):
    """Round 5: above 4096 rows the forward runs persistent workgroups with γ / β staged in LDS
    (ln_fwd_persist_kernel); its rows are bitwise the per-row kernel's (which a 4096-row call
    of the same first rows runs), statistics included, one LN or two."""
    torch.manual_seed(rows)
    x = torch.randn(rows, h, device=dev) * 2 + 0.5
    w1, b1 = torch.randn(h, device=dev), torch.randn(h, device=dev)
    w2, b2 = (torch.randn(h, device=dev), torch.randn(h, device=dev)) if dual else (None, None)

    def run(xx):
        n = xx.shape[0]
        y1 = torch.empty(n, h, device=dev, dtype=torch.bfloat16)
        y2 = torch.empty_like(y1) if dual else None
        mean, rstd = torch.empty(n, device=dev), torch.empty(n, device=dev)
        K.layernorm_fwd(xx, w1, b1, 1e-5, y1, mean, rstd, w2, b2, y2)
        return y1, y2, mean, rstd

    big = run(x)
    small = run(x[:4096].contiguous())
    for a, b in zip(big, small):
        if a is not None:
            assert torch.equal(a[:4096], b)
    r1 = torch.nn.functional.layer_norm(x, (h,), w1, b1, 1e-5)
    assert relerr(big[0], r1) < 4e-3


# ------------------------------------------------------------------ attention
def ref_attention(q, k, v, causal, scale):
    s = (q.float() @ k.float().transpose(-1, -2)) * scale
    if causal:
        S = q.shape[-2]
        s = s.masked_fill(torch.triu(torch.ones(S, S, device=q.device, dtype=torch.bool), 1), -math.inf)
    return torch.softmax(s, -1) @ v.float()


@pytest.mark.parametrize("D,causal,S,layout", [(256, True, 641, "interleaved"),  # S % 128 = 1:
                                                # waves whose keys all lie past S (clamped skip)
                                                (64, False, 197, "planar"), (256, True, 130, "interleaved"),
                                                (256, True, 70, "interleaved"), (128, False, 64, "planar"),
                                                (256, False, 200, "interleaved"),
                                                (64, True, 257, "interleaved"),
                                                # head dims run on the padded D = 128 kernels
                                                (80, True, 130, "interleaved"), (80, False, 77, "planar"),
                                                (96, True, 200, "interleaved"), (112, False, 64, "planar")])
def test_attention_fwd_bwd(K, D, causal, S, layout):
    torch.manual_seed(3)
    B, H = 2, 3
    T = B * S
    if layout == "interleaved":  # GPTNeoX: [t][h][3][D]
        hs, ps = 3 * D, D
    else:  # ViT fused qkv: [t][3][h][D]
        hs, ps = D, H * D
    qkv = bf(torch.randn(T, 3 * H * D, device=dev))

    def split(buf):
        v = buf.view(T, -1)
        parts = []
        for p in range(3):
            idx = torch.stack([torch.arange(D, device=dev) + h * hs + p * ps for h in range(H)])
            parts.append(v[:, idx].view(B, S, H, D).transpose(1, 2))
        return parts

    q, k, vv = split(qkv)
    scale = D ** -0.5
    out = torch.empty(T, H * D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * H * S, device=dev)
    K.attention_fwd(qkv, B, S, H, D, hs, ps, causal, scale, out, lse)
    qr, kr, vr = (t.float().clone().requires_grad_() for t in (q, k, vv))
    ref = ref_attention(qr, kr, vr, causal, scale)
    got = out.view(B, S, H, D).transpose(1, 2)
    assert relerr(got, ref) < 1e-2
    dout = bf(torch.randn(T, H * D, device=dev))
    ref.backward(dout.view(B, S, H, D).transpose(1, 2).float())
    dqkv = torch.zeros_like(qkv)
    K.attention_bwd(qkv, B, S, H, D, hs, ps, causal, scale, out, dout, lse, dqkv)
    dq, dk, dv = split(dqkv)
    assert relerr(dq, qr.grad) < 2e-2
    assert relerr(dk, kr.grad) < 2e-2
    assert relerr(dv, vr.grad) < 2e-2


@pytest.mark.parametrize("S,causal,G,B,Hk", [(707, True, 1, 2, 2), (641, True, 1, 2, 2), (300, False, 1, 2, 2),
                                          (300, True, 2, 2, 2),
                                          # the bench's persistent walk: 64 x 8 heads x 6 key
                                          # blocks = 3072 items, 12 per CU, so the next-item
                                          # prefetch under the epilogue runs on every CU
                                          (707, True, 1, 64, 8)])
def test_attention_dkdv_pair_bitwise_vs_ring(K, S, causal, G, B, Hk):
    """D = 256: the D-split wave-pair dK/dV kernel (MMPT_ATTN_PAIR=1, default) computes the same
    fp32 operations in the same order as the one-wave-per-SIMD ring kernel (P and dP cross LDS
    exactly): dQ, dK, dV and the dS tiles behind dQ bitwise equal."""
    from multimodal_llm_pretraining_amd import _lib

    torch.manual_seed(31)
    H, D = Hk * G, 256
    T = B * S
    qkv = bf(torch.randn(T, (H + 2 * Hk) * D, device=dev))
    out = torch.empty(T, H * D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * H * S, device=dev)
    K.attention_gqa_fwd(qkv, B, S, H, Hk, D, H * D, (H + Hk) * D, causal, D ** -0.5, out, lse)
    dout = bf(torch.randn(T, H * D, device=dev))
    got = {}
    prev = _lib.set_switch("MMPT_ATTN_PAIR", 1)
    try:
        for mode in (1, 0):
            _lib.set_switch("MMPT_ATTN_PAIR", mode)
            dqkv = torch.zeros_like(qkv)
            K.attention_gqa_bwd(qkv, B, S, H, Hk, D, H * D, (H + Hk) * D, causal, D ** -0.5, out,
                                dout, lse, dqkv)
            got[mode] = dqkv
    finally:
        _lib.set_switch("MMPT_ATTN_PAIR", prev)
    assert torch.equal(got[1], got[0])
    if B >= 64:  # forward, dQ and (round 5) dK / dV of sampled heads against
        # an fp32 reference — G = 1 here, so a kv head's gradient is its one query head's
        assert G == 1
        g = torch.Generator().manual_seed(5)
        for _ in range(3):
            b, h = int(torch.randint(B, (1,), generator=g)), int(torch.randint(H, (1,), generator=g))
            rows = slice(b * S, (b + 1) * S)
            kh = h // G
            q = qkv[rows, h * D:(h + 1) * D].float().requires_grad_()
            k = qkv[rows, (H + kh) * D:(H + kh + 1) * D].float().requires_grad_()
            v = qkv[rows, (H + Hk + kh) * D:(H + Hk + kh + 1) * D].float().requires_grad_()
            o = torch.nn.functional.scaled_dot_product_attention(q[None], k[None], v[None],
                                                                 is_causal=causal)[0]
            assert relerr(out[rows, h * D:(h + 1) * D], o) < 1e-2
            o.backward(dout[rows, h * D:(h + 1) * D].float())
            assert relerr(got[1][rows, h * D:(h + 1) * D], q.grad) < 2e-2
            assert relerr(got[1][rows, (H + kh) * D:(H + kh + 1) * D], k.grad) < 2e-2
            assert relerr(got[1][rows, (H + Hk + kh) * D:(H + Hk + kh + 1) * D], v.grad) < 2e-2


@pytest.mark.parametrize("D,S,causal,B,H", [(256, 707, True, 2, 2), (256, 300, False, 2, 2),
                                            (256, 707, True, 64, 8),  # persistent walk (bench)
                                            (128, 300, True, 2, 2)])  # the unfused fallback
def test_attention_bwd_rope_fused_bitwise(K, D, S, causal, B, H):
    """mmpt_attention_bwd_rope == mmpt_attention_bwd + mmpt_rope_inplace(inverse) on the q and k
    parts, bitwise: at D = 256 / 64 rotary dims the dK / dQ epilogues rotate (the same
    rounding, rope_rot), elsewhere the two kernels run in sequence."""
    from multimodal_llm_pretraining_amd.engine import rope_tables

    torch.manual_seed(47)
    T = B * S
    hs, ps = 3 * D, D
    rot = D // 4  # GPTNeoX rotary_pct 0.25
    cos, sin = (t.to(dev) for t in rope_tables(H * D, H, 0.25, 10000.0, S + 5))
    assert cos.shape[1] == rot
    qkv = bf(torch.randn(T, 3 * H * D, device=dev))
    dout = bf(torch.randn(T, H * D, device=dev))
    scale = D ** -0.5
    out = torch.empty(T, H * D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * H * S, device=dev)
    K.attention_fwd(qkv, B, S, H, D, hs, ps, causal, scale, out, lse)
    ref = torch.zeros_like(qkv)
    K.attention_bwd(qkv, B, S, H, D, hs, ps, causal, scale, out, dout, lse, ref)
    K.rope_inplace(ref, S, H, D, rot, hs, ps, cos, sin, inverse=True)
    got = torch.full_like(qkv, float("nan"))
    K.attention_bwd_rope(qkv, B, S, H, D, hs, ps, causal, scale, out, dout, lse, got, rot, cos, sin)
    assert torch.equal(got, ref)


@pytest.mark.parametrize("S,causal", [(707, True), (300, False)])
def test_attention_dq_recompute_path(K, S, causal):
    """D = 256 with MMPT_ATTN_DS=0 (the A/B path: dQ recomputed from Q, K, V, dO instead of read
    from the dS tiles; the slab LDS images feed both) against the default path and an fp32
    reference of dQ."""
    from multimodal_llm_pretraining_amd import _lib

    torch.manual_seed(43)
    B, H, D = 2, 2, 256
    T = B * S
    hs, ps = 3 * D, D
    qkv = bf(torch.randn(T, 3 * H * D, device=dev))
    dout = bf(torch.randn(T, H * D, device=dev))
    scale = D ** -0.5
    out = torch.empty(T, H * D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * H * S, device=dev)
    K.attention_fwd(qkv, B, S, H, D, hs, ps, causal, scale, out, lse)
    got = {}
    prev = _lib.set_switch("MMPT_ATTN_DS", 1)
    try:
        for mode in (1, 0):
            _lib.set_switch("MMPT_ATTN_DS", mode)
            dqkv = torch.zeros_like(qkv)
            K.attention_bwd(qkv, B, S, H, D, hs, ps, causal, scale, out, dout, lse, dqkv)
            got[mode] = dqkv
    finally:
        _lib.set_switch("MMPT_ATTN_DS", prev)
    assert relerr(got[0], got[1]) < 1e-2
    rows = slice(S, 2 * S)
    h = 1
    q, k, v = (qkv[rows, h * hs + i * ps:h * hs + i * ps + D].float().requires_grad_() for i in range(3))
    o = torch.nn.functional.scaled_dot_product_attention(q[None], k[None], v[None], is_causal=causal)[0]
    o.backward(dout[rows, h * D:(h + 1) * D].float())
    for i, ref in enumerate((q.grad, k.grad, v.grad)):
        assert relerr(got[0][rows, h * hs + i * ps:h * hs + i * ps + D], ref) < 2e-2


@pytest.mark.parametrize("S,causal,B,H", [(707, True, 2, 4), (300, False, 2, 4), (129, True, 3, 2),
                                          (707, True, 16, 32)])  # Pythia-2.8B heads, C5 sequence
def test_attention_native80_bitwise_vs_padded(K, S, causal, B, H):
    """head_dim 80 (Pythia-2.8B): the D = 128 kernels built to compute 80 dims (3 of 4 QK^T
    k-steps, 5 of 8 d-tiles; MMPT_ATTN_NATIVE80=1, default) against the same kernels over all
    128 dims with 80.. zero-filled (=0): the skipped products are exact zeros, so forward O,
    log-sum-exp and dQ/dK/dV are bitwise equal; the native forward and backward of one head
    also against an fp32 reference."""
    from multimodal_llm_pretraining_amd import _lib

    torch.manual_seed(41)
    D = 80
    T = B * S
    hs, ps = 3 * D, D  # GPTNeoX interleaved q|k|v per head
    qkv = bf(torch.randn(T, 3 * H * D, device=dev))
    dout = bf(torch.randn(T, H * D, device=dev))
    scale = D ** -0.5
    got = {}
    prev = _lib.set_switch("MMPT_ATTN_NATIVE80", 1)
    try:
        for mode in (1, 0):
            _lib.set_switch("MMPT_ATTN_NATIVE80", mode)
            out = torch.full((T, H * D), float("nan"), device=dev, dtype=torch.bfloat16)
            lse = torch.empty(B * H * S, device=dev)
            K.attention_fwd(qkv, B, S, H, D, hs, ps, causal, scale, out, lse)
            dqkv = torch.zeros_like(qkv)
            K.attention_bwd(qkv, B, S, H, D, hs, ps, causal, scale, out, dout, lse, dqkv)
            got[mode] = (out, lse, dqkv)
    finally:
        _lib.set_switch("MMPT_ATTN_NATIVE80", prev)
    for a, b in zip(got[1], got[0]):
        assert torch.equal(a, b)
    out, lse, dqkv = got[1]
    b, h = B - 1, H - 1
    rows = slice(b * S, (b + 1) * S)
    q, k, v = (qkv[rows, h * hs + i * ps:h * hs + i * ps + D].float().requires_grad_() for i in range(3))
    o = torch.nn.functional.scaled_dot_product_attention(q[None], k[None], v[None], is_causal=causal)[0]
    assert relerr(out[rows, h * D:(h + 1) * D], o) < 1e-2
    o.backward(dout[rows, h * D:(h + 1) * D].float())
    for i, ref in enumerate((q.grad, k.grad, v.grad)):
        assert relerr(dqkv[rows, h * hs + i * ps:h * hs + i * ps + D], ref) < 2e-2


def test_attention_deferred_max_rescale(K):
    """Rule-26 test for the deferred-max online softmax (attention.hip, THR = 8 in log2
    units): keys 100 / 300 / 600 carry growing spikes along a direction every query
    shares, so each query's running max jumps by >> THR at a LATE key block and the
    rescale branch must fire mid-sweep.  Full-tensor fp32 reference, elementwise."""
    torch.manual_seed(5)
    B, H, D, S = 1, 2, 256, 707
    T = B * S
    hs, ps = 3 * D, D
    qkv = torch.randn(T, 3 * H * D, device=dev)
    u = torch.randn(D, device=dev)
    u = u / u.norm()
    for h in range(H):
        qkv[:, h * hs:h * hs + D] += 2.0 * u
        for key, amp in ((100, 30.0), (300, 60.0), (600, 200.0)):
            qkv[key, h * hs + ps:h * hs + ps + D] += amp * u
    qkv = bf(qkv)
    v = qkv.view(T, H, 3, D)
    q, k, vv = (v[:, :, i].permute(1, 0, 2).unsqueeze(0).float() for i in range(3))
    scale = D ** -0.5
    out = torch.empty(T, H * D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * H * S, device=dev)
    K.attention_fwd(qkv, B, S, H, D, hs, ps, True, scale, out, lse)
    sc = (q @ k.transpose(-1, -2)) * scale
    mask = torch.ones(S, S, device=dev, dtype=torch.bool).tril()
    sc = sc.masked_fill(~mask, float("-inf"))
    ref = torch.softmax(sc, -1) @ vv
    got = out.view(B, S, H, D).transpose(1, 2).float()
    err = (got - ref).abs().max().item()
    assert err < 3e-2 * ref.abs().max().item(), err
    ref_lse = torch.logsumexp(sc, -1).reshape(-1)
    assert (lse - ref_lse).abs().max().item() < 1e-3 * ref_lse.abs().max().item()
    # the data really exercises the rescale: row 650's max jumps by > THR (8, log2
    # units) at key 600, i.e. in key block 9 of the sweep
    l2e = 1.4426950408889634
    jump = (sc[0, :, 650, 600] - sc[0, :, 650, :600].max(-1).values) * l2e
    assert (jump > 8).all(), jump


@pytest.mark.parametrize("rot", [64, 20, 10])  # 16-B vector path / pair kernel (two / one pairs)
def test_rope_roundtrip(K, rot):
    torch.manual_seed(4)
    S, H, D = 50, 2, 256
    T = 2 * S
    qkv = bf(torch.randn(T, H * 3 * D, device=dev))
    inv = 1.0 / (10000 ** (torch.arange(0, rot, 2, dtype=torch.float) / rot))
    fr = torch.arange(S, dtype=torch.float)[:, None] * inv[None]
    emb = torch.cat([fr, fr], -1)
    cos, sin = emb.cos().to(dev).contiguous(), emb.sin().to(dev).contiguous()
    x = qkv.clone()
    K.rope_inplace(x, S, H, D, rot, 3 * D, D, cos, sin)
    v = qkv.view(T, H, 3, D).float()
    pos = torch.arange(T, device=dev) % S
    c, s_ = cos[pos][:, None, :], sin[pos][:, None, :]
    for p in (0, 1):
        r = v[:, :, p, :rot]
        rh = torch.cat([-r[..., rot // 2:], r[..., :rot // 2]], -1)
        ref = torch.cat([r * c + rh * s_, v[:, :, p, rot:]], -1)
        assert relerr(x.view(T, H, 3, D)[:, :, p], ref) < 4e-3
    assert torch.equal(x.view(T, H, 3, D)[:, :, 2], qkv.view(T, H, 3, D)[:, :, 2])
    if (rot // 2) % 8 != 0:
        # an even rotary half on 4-B aligned rows runs rope_pair_kernel<2> (two pairs per
        # thread, 4-B accesses); a 2-B aligned view of the same rows forces <1>: bitwise equal
        xp = torch.zeros(T, H * 3 * D + 2, device=dev, dtype=torch.bfloat16)
        xp[:, 1:1 + H * 3 * D] = qkv
        K.rope_inplace(xp, S, H, D, rot, 3 * D, D, cos, sin, offset=1)
        assert torch.equal(xp[:, 1:1 + H * 3 * D], x)
    # inverse of forward is the identity up to bf16 rounding
    K.rope_inplace(x, S, H, D, rot, 3 * D, D, cos, sin, inverse=True)
    assert relerr(x, qkv) < 8e-3


# ------------------------------------------------------------------ loss / reductions
def test_cross_entropy(K):
    torch.manual_seed(5)
    R, V = 37, 50304
    logits = bf(torch.randn(R, V, device=dev) * 3)
    labels = torch.randint(0, V, (R,), device=dev)
    labels[::5] = -100
    n = (labels != -100).sum().item()
    loss_rows = torch.empty(R, device=dev)
    dl = torch.empty_like(logits)
    K.cross_entropy(logits, labels, -100, 1.0 / n, loss_rows, dl)
    x = logits.float().requires_grad_()
    ref = torch.nn.functional.cross_entropy(x, labels, ignore_index=-100)
    ref.backward()
    tot = torch.empty(1, device=dev)
    K.sum_f32(loss_rows, tot)
    assert abs(tot.item() / n - ref.item()) < 1e-4
    assert relerr(dl, x.grad) < 5e-3


@pytest.mark.parametrize("V,vv,inplace", [(50304, 50304, False), (50304, 50304, True),
                                           (2048, 2000, True), (128264, 128257, False)])
def test_cross_entropy_register_row_bitwise(K, V, vv, inplace):
    """The register-resident cross entropy (the row read once; MMPT_CE_REG) is bitwise the
    two-pass kernel — same chunk-per-thread assignment, so the same online max / sum order —
    for the loss rows and every gradient, in place (dlogits over logits, the engine's form:
    the label's logit comes from registers) and not, with padded vocabulary columns and
    ignored rows; vocabularies past 65,536 keep the two-pass kernel."""
    from multimodal_llm_pretraining_amd import _lib

    torch.manual_seed(6)
    R = 41
    logits = bf(torch.randn(R, V, device=dev) * 3)
    labels = torch.randint(0, vv, (R,), device=dev)
    labels[::5] = -100

    def run():
        x = logits.clone()
        loss = torch.empty(R, device=dev)
        dl = x if inplace else torch.empty_like(x)
        _lib.call("mmpt_cross_entropy", R, V, vv, x.data_ptr(), V, labels.data_ptr(), -100, 0.5,
                  loss.data_ptr(), dl.data_ptr(), V, torch.cuda.current_stream().cuda_stream)
        return loss, dl

    prev = _lib.set_switch("MMPT_CE_REG", 0)
    try:
        l0, d0 = run()
        _lib.set_switch("MMPT_CE_REG", 1)
        l1, d1 = run()
    finally:
        _lib.set_switch("MMPT_CE_REG", prev)
    assert torch.equal(l0, l1)
    assert torch.equal(d0.view(torch.int16), d1.view(torch.int16))
    ref = torch.nn.functional.cross_entropy(logits.float()[:, :vv], labels, ignore_index=-100,
                                            reduction="none")
    assert (l1 - ref).abs().max().item() < 1e-4


def test_sums(K):
    x = torch.randn(1_000_003, device=dev)
    o = torch.empty(1, device=dev)
    K.sum_f32(x, o)
    assert abs(o.item() - x.double().sum().item()) < 1e-2
    K.sumsq_f32(x, o)
    assert abs(o.item() / (x.double() ** 2).sum().item() - 1) < 1e-5


@pytest.mark.parametrize("rows,cols", [(1234, 3072), (45248, 2048), (7, 8)])
def test_colsum(K, rows, cols):
    dy = bf(torch.randn(rows, cols, device=dev))
    out = torch.ones(cols, device=dev)
    out2 = torch.full((cols,), 2.0, device=dev)
    K.colsum(dy, out, accumulate=True, dbias2=out2)
    ref = bf(dy.float().sum(0)).float()
    assert relerr(out - 1, ref) < 5e-3 and relerr(out2 - 2, ref) < 5e-3


# ------------------------------------------------------------------ embeddings / glue
def test_embed_merge(K):
    torch.manual_seed(6)
    V, h, rows = 100, 64, 40
    table = torch.randn(V, h, device=dev)
    ids = torch.randint(0, V, (rows,), device=dev)
    img_map = torch.full((rows,), -1, dtype=torch.int32, device=dev)
    img_map[3:9] = torch.arange(6, dtype=torch.int32, device=dev)
    img = bf(torch.randn(6, h, device=dev))
    out = torch.empty(rows, h, device=dev)
    K.embed_fwd(ids, table, out, img_map, img)
    ref = table[ids].clone()
    ref[3:9] = img.float()
    assert torch.equal(out, ref)
    dout = torch.randn(rows, h, device=dev)
    dtab = torch.zeros(V, h, device=dev)
    dimg = torch.empty(6, h, device=dev, dtype=torch.bfloat16)
    K.embed_bwd(_segments(ids, img_map), dout, dtab, img_map, dimg)
    d2 = dout.clone()
    d2[3:9] = 0
    ref_t = torch.zeros(V, h, device=dev).index_add_(0, ids, d2)
    assert relerr(dtab, ref_t) < 1e-6
    assert torch.equal(dimg, bf(dout[3:9]))


def _segments(ids, img_map=None):
    import numpy as np

    from multimodal_llm_pretraining_amd.engine import sort_segments

    idn = ids.cpu().numpy()
    rows = np.arange(idn.size) if img_map is None else np.flatnonzero(img_map.cpu().numpy() < 0)
    return tuple(torch.from_numpy(a).to(dev) for a in sort_segments(idn, rows))


@pytest.mark.parametrize("V,rows,h", [(4, 8192, 512), (50304, 45248, 2048), (1, 300, 8)])
def test_embed_bwd_deterministic_collisions(K, V, rows, h):
    """K8/P3: the sorted segmented reduction is bitwise repeatable and equals the same
    position-ordered fp32 sum on the host, however many rows share an id (V = 4: ~2000
    rows per id; V = 1: every row collides)."""
    import numpy as np

    torch.manual_seed(11)
    ids = torch.randint(0, V, (rows,), device=dev)
    dout = torch.randn(rows, h, device=dev)
    seg = _segments(ids)
    base = torch.randn(V, h, device=dev)
    outs = []
    for _ in range(3):
        dtab = base.clone()
        K.embed_bwd(seg, dout, dtab)
        outs.append(dtab)
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    # host restatement in the same order: acc = Σ_rows-of-id (position order); tab += acc
    idn, dn = ids.cpu().numpy(), dout.cpu().numpy()
    ref = base.cpu().numpy().copy()
    for v in np.unique(idn)[:64]:
        acc = np.zeros(h, np.float32)
        for r in np.flatnonzero(idn == v):
            acc += dn[r]
        ref[v] += acc
        assert np.array_equal(outs[0][int(v)].cpu().numpy(), ref[v]), int(v)


def test_patch_embed_glue(K):
    torch.manual_seed(7)
    B, C, S, p, h = 2, 3, 64, 16, 96
    np_ = (S // p) ** 2
    pix = torch.rand(B, C, S, S, device=dev)
    cols = torch.empty(B * np_, C * p * p, device=dev, dtype=torch.bfloat16)
    K.im2col(pix, p, cols)
    ref = bf(pix).unfold(2, p, p).unfold(3, p, p)  # B C gy gx p p
    ref = ref.permute(0, 2, 3, 1, 4, 5).reshape(B * np_, C * p * p)
    assert torch.equal(cols, ref)
    patch = bf(torch.randn(B * np_, h, device=dev))
    cls, pos = torch.randn(h, device=dev), torch.randn(np_ + 1, h, device=dev)
    out = torch.empty(B * (np_ + 1), h, device=dev)
    K.vit_embed_fwd(B, np_, patch, cls, pos, out)
    ref = torch.cat([cls.expand(B, 1, h), patch.float().view(B, np_, h)], 1) + pos
    assert torch.equal(out.view(B, np_ + 1, h), ref)
    dout = torch.randn(B * (np_ + 1), h, device=dev)
    dcls, dpos = torch.zeros(h, device=dev), torch.zeros(np_ + 1, h, device=dev)
    dpatch = torch.empty_like(patch)
    K.vit_embed_bwd(B, np_, dout, dcls, dpos, dpatch)
    d3 = dout.view(B, np_ + 1, h)
    assert relerr(dcls, d3[:, 0].sum(0)) < 1e-6 and relerr(dpos, d3.sum(0)) < 1e-6
    assert torch.equal(dpatch, bf(d3[:, 1:].reshape(-1, h)))
    sel = torch.empty(B * np_, h, device=dev, dtype=torch.bfloat16)
    K.select_patches_fwd(B, np_, out, sel)
    assert torch.equal(sel, bf(out.view(B, np_ + 1, h)[:, 1:].reshape(-1, h)))
    dx = torch.full((B * (np_ + 1), h), 2.0, device=dev)
    K.select_patches_bwd(B, np_, sel, dx, True)
    exp = torch.full((B, np_ + 1, h), 2.0, device=dev)
    exp[:, 1:] += sel.float().view(B, np_, h)
    assert torch.equal(dx.view(B, np_ + 1, h), exp)


# ------------------------------------------------------------------ optimizer
@pytest.mark.parametrize("adamw,wd", [(False, 0.0), (True, 0.1), (False, 0.01)])
def test_adam_matches_torch(K, adamw, wd):
    torch.manual_seed(8)
    n = 4096 + 4
    p0 = torch.randn(n, device=dev)
    p_ref = p0.clone().requires_grad_()
    opt = (torch.optim.AdamW if adamw else torch.optim.Adam)([p_ref], lr=1e-3, betas=(0.9, 0.95),
                                                            eps=1e-8, weight_decay=wd, foreach=False)
    p, m, v = p0.clone(), torch.zeros(n, device=dev), torch.zeros(n, device=dev)
    pb = torch.empty(n, device=dev, dtype=torch.bfloat16)
    for step in range(1, 4):
        g = torch.randn(n, device=dev)
        p_ref.grad = g.clone()
        opt.step()
        K.adam_step(p, g, m, v, pb, lr=1e-3, beta1=0.9, beta2=0.95, eps=1e-8, weight_decay=wd,
                    adamw=adamw, step=step)
    assert (p - p_ref.detach()).abs().max().item() < 1e-6
    assert torch.equal(pb, bf(p))


@pytest.mark.parametrize("rows,cols", [(2048, 6144), (72, 8), (768, 3072)])
def test_transpose(K, rows, cols):
    x = bf(torch.randn(rows, cols, device=dev))
    y = torch.empty(cols, rows, device=dev, dtype=torch.bfloat16)
    K.transpose_bf16(x, y)
    assert torch.equal(y, x.t())


def test_clip_coef(K):
    s = torch.tensor([16.0], device=dev)
    c = torch.empty(1, device=dev)
    K.clip_coef(s, 1.0, c)
    assert abs(c.item() - 1.0 / (4.0 + 1e-6)) < 1e-7


# ------------------------------------------------------------------ Llama side (K17)
@pytest.mark.parametrize("rows,h", [(3000, 2048), (37, 256)])
def test_rmsnorm(K, rows, h):
    """LlamaRMSNorm fwd (fp32 stats, w * x̂ -> bf16) and bwd (dx with residual add + bf16
    copy, dw) vs torch fp32 autograd of HF's formula."""
    torch.manual_seed(21)
    x = torch.randn(rows, h, device=dev) * 3 + 0.2
    w = torch.rand(h, device=dev) + 0.5
    y = torch.empty(rows, h, device=dev, dtype=torch.bfloat16)
    rstd = torch.empty(rows, device=dev)
    K.rmsnorm_fwd(x, w, 1e-5, y, rstd)
    xr, wr = x.clone().requires_grad_(), w.clone().requires_grad_()
    ref = wr * (xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-5))
    d = (y.float() - bf(ref.detach()).float()).abs()
    assert (d <= 2.0 ** -7 * ref.detach().abs() + 1e-30).all()  # within one bf16 rounding
    assert relerr(rstd, torch.rsqrt(x.pow(2).mean(-1) + 1e-5)) < 1e-6
    dy = bf(torch.randn(rows, h, device=dev))
    ref.backward(dy.float())
    resid = torch.randn(rows, h, device=dev)
    dx = resid.clone()
    dxb = torch.empty(rows, h, device=dev, dtype=torch.bfloat16)
    dw = torch.ones(h, device=dev)
    K.rmsnorm_bwd(x, rstd, dy, w, dx, dw=dw, dresid=dx, dx_bf16=dxb)
    assert relerr(dx - resid, xr.grad) < 1e-5
    assert torch.equal(dxb, bf(dx))
    assert relerr(dw - 1, wr.grad) < 1e-5


@pytest.mark.parametrize("S,causal,H,Hk,D", [(300, True, 8, 2, 64), (1087, True, 32, 8, 64),
                                             (129, False, 4, 4, 64), (577, True, 4, 1, 64),
                                             (300, True, 4, 2, 256), (200, False, 4, 1, 256)])
def test_gqa_attention(K, S, causal, H, Hk, D):
    """Llama-3 GQA (D = 64; D = 256 runs the wave-pair dK/dV kernel's query-head sweep) on the
    fused [q (H heads) | k (Hk) | v (Hk)] projection output vs fp32 softmax attention with
    repeat_kv; dK/dV summed over each group."""
    torch.manual_seed(22)
    B = 2
    T = B * S
    qkv = bf(torch.randn(T, (H + 2 * Hk) * D, device=dev))
    q = qkv[:, :H * D].view(B, S, H, D).transpose(1, 2)
    k = qkv[:, H * D:(H + Hk) * D].view(B, S, Hk, D).transpose(1, 2)
    v = qkv[:, (H + Hk) * D:].view(B, S, Hk, D).transpose(1, 2)
    qr, kr, vr = (t.float().clone().requires_grad_() for t in (q, k, v))
    G = H // Hk
    ref = ref_attention(qr, kr.repeat_interleave(G, 1), vr.repeat_interleave(G, 1), causal, D ** -0.5)
    out = torch.empty(T, H * D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * H * S, device=dev)
    K.attention_gqa_fwd(qkv, B, S, H, Hk, D, H * D, (H + Hk) * D, causal, D ** -0.5, out, lse)
    assert relerr(out.view(B, S, H, D).transpose(1, 2), ref) < 1e-2
    dout = bf(torch.randn(T, H * D, device=dev))
    ref.backward(dout.view(B, S, H, D).transpose(1, 2).float())
    dqkv = torch.zeros_like(qkv)
    K.attention_gqa_bwd(qkv, B, S, H, Hk, D, H * D, (H + Hk) * D, causal, D ** -0.5, out, dout,
                        lse, dqkv)
    dq = dqkv[:, :H * D].view(B, S, H, D).transpose(1, 2)
    dk = dqkv[:, H * D:(H + Hk) * D].view(B, S, Hk, D).transpose(1, 2)
    dv = dqkv[:, (H + Hk) * D:].view(B, S, Hk, D).transpose(1, 2)
    assert relerr(dq, qr.grad) < 2e-2
    assert relerr(dk, kr.grad) < 2e-2
    assert relerr(dv, vr.grad) < 2e-2


@pytest.mark.parametrize("M,F", [(333, 128), (4104, 1024)])
def test_swiglu_epilogues(K, M, F):
    """SwiGLU fwd (blocked gate|up GEMM -> pre-activations + bf16(bf16(silu(g)) * u)) and
    bwd (act-gradient GEMM -> d gate, d up) against torch running the same bf16 ops on the
    CPU (the oracle's autocast semantics); ≥ 99.5% bit-exact, ≤ 1 bf16 ulp elsewhere."""
    from oracle.model import block_gate_up

    torch.manual_seed(23)
    h = 256
    x = bf(torch.randn(M, h, device=dev))
    wg, wu = bf(torch.randn(F, h, device=dev) * 0.1), bf(torch.randn(F, h, device=dev) * 0.1)
    w = block_gate_up(wg, wu).contiguous()
    gu = torch.empty(M, 2 * F, device=dev, dtype=torch.bfloat16)
    act = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
    K.gemm(x, w, gu, epilogue=K.EPI_BF16_SWIGLU, out2=act)
    g_ref = bf(x.float() @ wg.float().t())
    u_ref = bf(x.float() @ wu.float().t())
    from oracle.model import unblock_gate_up
    g_got, u_got = unblock_gate_up(gu.t(), F)
    assert relerr(g_got.t(), g_ref) < 5e-3 and relerr(u_got.t(), u_ref) < 5e-3

    def close(got, ref, frac=0.995):
        dd = (got.cpu().float() - ref.float()).abs()
        ulp = ref.float().abs().clamp_min(1e-30) * 2.0 ** -7
        return (dd == 0).float().mean().item() >= frac and bool((dd <= ulp + 1e-30).all())

    gc, uc = g_got.t().cpu(), u_got.t().cpu()  # the GEMM's own bf16 gate/up
    a_ref = torch.nn.functional.silu(gc) * uc  # bf16 CPU ops, as under autocast
    assert close(act, a_ref)
    # backward: d act = bf16(dY @ W_down) produced by the GEMM; (dg, du) by autograd (CPU bf16)
    wd = bf(torch.randn(h, F, device=dev) * 0.1)
    dy = bf(torch.randn(M, h, device=dev))
    wdt = wd.t().contiguous()  # [F, h]: the transposed shadow the engine passes
    dgu = torch.empty(M, 2 * F, device=dev, dtype=torch.bfloat16)
    K.gemm(dy, wdt, dgu, epilogue=K.EPI_BF16_DSWIGLU, aux=gu)
    dact = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
    K.gemm(dy, wdt, dact)  # the same accumulation, plain epilogue
    gr, ur = gc.clone().requires_grad_(), uc.clone().requires_grad_()
    (torch.nn.functional.silu(gr) * ur).backward(dact.cpu())
    dg_got, du_got = unblock_gate_up(dgu.t(), F)
    assert close(dg_got.t(), gr.grad) and close(du_got.t(), ur.grad)


@pytest.mark.parametrize("M", [8192, 65536])  # gemm128 (K = 8) and gemm4p (K = 64) epilogue paths
def test_gelu_epilogues_every_bf16_input(K, M):
    """GELU and dGELU epilogues on every finite bf16 input with |x| <= 20 (the whole range a
    bf16 pre-activation can usefully take): out = x·1 through the GEMM, then GELU(x) and
    bf16(1 · GELU'(x)) against the fp64 erfc-GELU rounded to bf16.  Measured: GELU bitwise equal
    on every input; dGELU bitwise equal except x = -13.25, -13.3125 (exact 4e-38 / 2e-38, kernel
    0: exp(-x²/2) is an fp32 denormal there)."""
    import math

    bits = torch.arange(0, 1 << 16, dtype=torch.int32).to(torch.int16)
    xs = bits.view(torch.bfloat16).float()
    xs = xs[torch.isfinite(xs) & (xs.abs() <= 20)]
    n = xs.numel()
    reps = -(-M // n)
    xs = xs.repeat(reps)[:M]
    A = torch.zeros(M, 8 if M == 8192 else 64, device=dev, dtype=torch.bfloat16)
    A[:, 0] = xs.to(dev).to(torch.bfloat16)
    W = torch.zeros(8 if M == 8192 else 256, 8 if M == 8192 else 64, device=dev, dtype=torch.bfloat16)
    W[0, 0] = 1.0
    pre = torch.empty(M, W.shape[0], device=dev, dtype=torch.bfloat16)
    act = torch.empty_like(pre)
    K.gemm(A, W, pre, epilogue=K.EPI_BF16_GELU, out2=act)
    x64 = xs.double()
    # Φ(x) = erfc(-x/√2)/2: 1 + erf(x/√2) cancels catastrophically for x << 0, even in fp64
    ref = 0.5 * x64 * torch.special.erfc(-x64 / math.sqrt(2.0))
    got = act[:, 0].float().cpu()
    assert torch.equal(pre[:, 0].float().cpu(), xs)
    tiny = ref.abs() < 1.2e-38
    bad = (got != ref.float().to(torch.bfloat16).float()) & ~tiny
    assert bad.sum().item() == 0, (xs[bad][:8], got[bad][:8], ref[bad][:8])
    # dGELU: incoming gradient 1 (A = 1 in column 0), aux = x
    ones = torch.zeros(M, 8 if M == 8192 else 64, device=dev, dtype=torch.bfloat16)
    ones[:, 0] = 1.0
    aux = torch.zeros(M, W.shape[0], device=dev, dtype=torch.bfloat16)
    aux[:, 0] = xs.to(dev).to(torch.bfloat16)
    dg = torch.empty_like(pre)
    K.gemm(ones, W, dg, epilogue=K.EPI_BF16_DGELU, aux=aux)
    dref = 0.5 * torch.special.erfc(-x64 / math.sqrt(2.0)) + x64 * torch.exp(-0.5 * x64 * x64) / math.sqrt(2 * math.pi)
    dgot = dg[:, 0].float().cpu()
    # exp(-x²/2) of |x| > 13.2 is an fp32 denormal the hardware exp flushes: the exact
    # derivative there is below 1e-37 and the kernel returns 0
    dbad = (dgot != dref.float().to(torch.bfloat16).float()) & ~(dref.abs() < 1e-37)
    # the fp32 evaluation of Φ(x) + x·φ(x) may land on the other side of a bf16 rounding
    # boundary: allow a handful of 1-ulp cases, nothing worse
    ulp = (dref.float().to(torch.bfloat16).float() - dgot).abs() <= 2.0 ** -7 * dref.abs().float() + 1e-38
    assert dbad.sum().item() <= 8 and bool(ulp[dbad].all()), (xs[dbad][:8], dgot[dbad][:8], dref[dbad][:8])


@pytest.mark.parametrize("n,parts", [(1000, 3), (256, 1), (4096, 2)])
def test_zeropp_quant_kernels_match_oracle(K, n, parts):
    """ZeRO++ qwZ / qgZ kernels against oracle/quant.py: int8 / int4 codes and scales bitwise,
    the int8 dequantization bitwise after the bf16 rounding, the int4 dequantize-and-sum
    within fp32 rounding (the kernel fuses q·s + acc).  Includes a partial last block
    (n = 1000) and an all-zero block (scale 0, codes 0)."""
    import numpy as np

    from oracle import quant as Q

    torch.manual_seed(5)
    x = torch.randn(parts * n) * torch.linspace(0.01, 3.0, parts * n)
    x[:256] = 0.0  # a zero block
    xb = bf(x.to(dev))
    q8 = torch.empty(parts * n, dtype=torch.int8, device=dev)
    s8 = torch.empty(parts * K.quant_blocks(n), device=dev)
    K.quant_int8(xb, parts, q8, s8)
    rq, rs = Q.quant_int8(xb.float().cpu().numpy(), parts)
    assert np.array_equal(q8.cpu().numpy(), rq)
    assert np.array_equal(s8.cpu().numpy(), rs)
    y = torch.empty_like(xb)
    K.dequant_int8(q8, s8, parts, y)
    want = torch.from_numpy(Q.dequant_int8(rq, rs, parts)).to(torch.bfloat16)
    assert torch.equal(y.cpu(), want)
    # |x - dequant(x)| <= scale/2 + the bf16 rounding of the result
    sc = s8.view(parts, -1).repeat_interleave(256, dim=1)[:, :n].reshape(-1)
    assert ((y.float() - xb.float()).abs() <= 0.5 * sc + 2 ** -8 * xb.float().abs() + 1e-30).all()
    # int4 gradients
    g = x.to(dev)
    q4 = torch.empty(parts * n // 2, dtype=torch.uint8, device=dev)
    s4 = torch.empty(parts * K.quant_blocks(n), device=dev)
    K.quant_int4(g, parts, q4, s4)
    rq4, rs4 = Q.quant_int4(g.cpu().numpy(), parts)
    assert np.array_equal(q4.cpu().numpy(), rq4)
    assert np.array_equal(s4.cpu().numpy(), rs4)
    acc = torch.full((n,), 0.25, device=dev)
    K.dequant_int4_sum(q4, s4, parts, acc)
    ref = Q.dequant_int4_sum(rq4, rs4, parts) + np.float32(0.25)
    torch.testing.assert_close(acc.cpu(), torch.from_numpy(ref), rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("M", [8192, 65536])  # gemm128 (K = 8) and gemm4p (K = 64, packed rows + fixup)
def test_gelu_epilogues_non_finite(K, M):
    """GELU / dGELU epilogues outside the tables, against the erf form the reference's GPU
    GELU evaluates (x * 0.5 * erfc(-x / sqrt 2), backward cdf + x * pdf; fp64 here): nan
    stays nan, GELU(+inf) = +inf, GELU(-inf) = nan (-inf * 0), GELU'(+-inf) = nan (inf * 0),
    |x| >= 32 gives the limits (x / -0, 1 / 0).  (torch's vectorised CPU GELU returns nan
    for +inf as well.)  A non-finite value lands in rows otherwise full of table values, so
    the packed rows' wave-uniform fixup is exercised."""
    import math

    special = torch.tensor([float("nan"), float("inf"), -float("inf"), 32.0, -32.0, 1e30, -1e30,
                            3.0e38, -3.0e38, 40.0, -40.0])
    xs = (torch.rand(M) * 8 - 4).to(torch.bfloat16).float()
    pos = torch.arange(0, M, 97)[: 4 * special.numel()]
    xs[pos] = special.repeat(4)[: pos.numel()]
    x64 = xs.double()
    ref = 0.5 * x64 * torch.special.erfc(-x64 / math.sqrt(2.0))
    dref = 0.5 * torch.special.erfc(-x64 / math.sqrt(2.0)) + \
        x64 * torch.exp(-0.5 * x64 * x64) / math.sqrt(2 * math.pi)
    W = torch.zeros(8 if M == 8192 else 256, 8 if M == 8192 else 64, device=dev, dtype=torch.bfloat16)
    W[0, 0] = 1.0
    A = torch.zeros(M, 8 if M == 8192 else 64, device=dev, dtype=torch.bfloat16)
    A[:, 0] = xs.to(dev).to(torch.bfloat16)
    pre = torch.empty(M, W.shape[0], device=dev, dtype=torch.bfloat16)
    act = torch.empty_like(pre)
    K.gemm(A, W, pre, epilogue=K.EPI_BF16_GELU, out2=act)
    got = act[:, 0].float().cpu()
    want = ref.float().to(torch.bfloat16).float()
    assert torch.equal(torch.isnan(got), torch.isnan(want)), (xs[torch.isnan(got) != torch.isnan(want)])
    fin = ~torch.isnan(want)
    assert torch.equal(got[fin], want[fin]), (xs[fin][got[fin] != want[fin]][:8])
    assert torch.equal(torch.signbit(got[fin]), torch.signbit(want[fin]))  # GELU(-40) = -0
    ones = torch.zeros(M, 8 if M == 8192 else 64, device=dev, dtype=torch.bfloat16)
    ones[:, 0] = 1.0
    aux = torch.zeros(M, W.shape[0], device=dev, dtype=torch.bfloat16)
    aux[:, 0] = xs.to(dev).to(torch.bfloat16)
    dg = torch.empty_like(pre)
    K.gemm(ones, W, dg, epilogue=K.EPI_BF16_DGELU, aux=aux)
    dgot = dg[:, 0].float().cpu()
    dwant = dref.float().to(torch.bfloat16).float()
    assert torch.equal(torch.isnan(dgot), torch.isnan(dwant)), (xs[torch.isnan(dgot) != torch.isnan(dwant)])
    big = xs.abs() >= 32
    assert torch.equal(dgot[big & ~torch.isnan(dwant)], dwant[big & ~torch.isnan(dwant)])


def _all_bf16_rows(M):
    """every finite bf16 value once (65,280), cycled to M rows"""
    bits = torch.arange(0, 1 << 16, dtype=torch.int32).to(torch.int16)
    xs = bits.view(torch.bfloat16).float()
    xs = xs[torch.isfinite(xs)]
    return xs.repeat(-(-M // xs.numel()))[:M].to(torch.bfloat16)


def _ulp_close(got, want, floor=1e-36):
    """bitwise equal, except values below `floor` in magnitude (fp32 exp underflow in either
    evaluation: x in [-52, -51.5] gives quick-GELU values near 5e-37 on the CPU and 0 from the
    device's exp) and at most 1 bf16 ulp on ≤ 0.01% of the rest"""
    g, w = got.float().cpu(), want.float().cpu()
    both_nan = torch.isnan(g) & torch.isnan(w)
    diff = (g != w) & ~both_nan & ~((g.abs() < floor) & (w.abs() < floor))
    ulp = (g - w).abs() <= 2.0 ** -7 * w.abs() + 1e-38
    idx = diff.nonzero().flatten()[:8]
    return (diff.float().mean().item() <= 1e-4 and bool(ulp[diff].all()),
            (int(diff.sum()), idx.tolist(), g[idx].tolist(), w[idx].tolist()))


def test_gemm4p_activation_tables_every_bf16_input(K):
    """Round 5: quick-GELU (CLIP) and SwiGLU (Llama) forms on gemm4p — the forwards from the
    host-built tables (g_qgelu_lut / g_silu_lut, out-of-table values through the general code),
    the backwards through the general epilogue — on EVERY finite bf16 input, against torch
    running the same bf16 ops on the CPU (the oracle's autocast semantics).  Measured: bitwise
    except 3 outputs below 1e-36 (CPU and device fp32 exp underflow differently; the formula
    path of the retired gemm256 kernel gave the same 3, profiles/r05/act4p/)."""
    M = 65536  # 256 tile rows x 1 tile column: the big-tile (gemm4p) path
    xs = _all_bf16_rows(M)
    torch.manual_seed(31)
    other = (torch.randn(M) * 2).to(torch.bfloat16)  # up values / incoming gradients
    # quick-GELU forward: column 0 of pre = x (A[:, 0] = x, W[0, 0] = 1), K = 64
    A = torch.zeros(M, 64, dtype=torch.bfloat16)
    A[:, 0] = xs
    A[:, 1] = other
    A = A.to(dev)
    W = torch.zeros(256, 64, device=dev, dtype=torch.bfloat16)
    W[0, 0] = 1.0
    pre = torch.empty(M, 256, device=dev, dtype=torch.bfloat16)
    act = torch.empty_like(pre)
    K.gemm(A, W, pre, epilogue=K.EPI_BF16_QGELU, out2=act)
    assert K.gemm_last_kernel().startswith("gemm4p_kernel"), K.gemm_last_kernel()
    assert torch.equal(pre[:, 0].cpu(), xs)
    want = xs * torch.sigmoid(1.702 * xs)  # bf16 CPU ops, as under autocast
    ok, nd = _ulp_close(act[:, 0], want)
    assert ok, ("qgelu", nd, xs[nd[1]].tolist())
    # dQGELU (general epilogue): incoming gradient d = A[:, 1] (W2[0, 1] = 1), aux = x
    W2 = torch.zeros(256, 64, device=dev, dtype=torch.bfloat16)
    W2[0, 1] = 1.0
    dg = torch.empty_like(pre)
    K.gemm(A, W2, dg, epilogue=K.EPI_BF16_DQGELU, aux=pre)
    assert K.gemm_last_kernel().startswith("gemm4p_kernel"), K.gemm_last_kernel()
    x = xs.clone().requires_grad_()
    (x * torch.sigmoid(1.702 * x)).backward(other)
    ok, nd = _ulp_close(dg[:, 0], x.grad)
    assert ok, ("dqgelu", nd, xs[nd[1]].tolist(), other[nd[1]].tolist())
    # SwiGLU forward: blocked gate|up weight [256, 64] (gate rows 0-127, their up rows 128-255):
    # gate feature 0 = x, up feature 0 = other
    Wg = torch.zeros(256, 64, device=dev, dtype=torch.bfloat16)
    Wg[0, 0] = 1.0
    Wg[128, 1] = 1.0
    gu = torch.empty(M, 256, device=dev, dtype=torch.bfloat16)
    sact = torch.empty(M, 128, device=dev, dtype=torch.bfloat16)
    K.gemm(A, Wg, gu, epilogue=K.EPI_BF16_SWIGLU, out2=sact)
    assert K.gemm_last_kernel().startswith("gemm4p_kernel"), K.gemm_last_kernel()
    assert torch.equal(gu[:, 0].cpu(), xs) and torch.equal(gu[:, 128].cpu(), other)
    assert not gu[:, 1:128].cpu().any() and not sact[:, 1:].cpu().any()
    want = torch.nn.functional.silu(xs) * other
    ok, nd = _ulp_close(sact[:, 0], want)
    assert ok, ("swiglu", nd, xs[nd[1]].tolist(), other[nd[1]].tolist())
    # dSwiGLU (general epilogue): d act = A[:, 1] through wdt [F = 128, 64] (row 0, column 1)
    wdt = torch.zeros(128, 64, device=dev, dtype=torch.bfloat16)
    wdt[0, 1] = 1.0
    dgu = torch.empty(M, 256, device=dev, dtype=torch.bfloat16)
    K.gemm(A, wdt, dgu, epilogue=K.EPI_BF16_DSWIGLU, aux=gu)
    assert K.gemm_last_kernel().startswith("gemm4p_kernel"), K.gemm_last_kernel()
    gr, ur = xs.clone().requires_grad_(), other.clone().requires_grad_()
    (torch.nn.functional.silu(gr) * ur).backward(other)
    ok, nd = _ulp_close(dgu[:, 0], gr.grad)
    assert ok, ("dswiglu gate", nd, xs[nd[1]].tolist(), other[nd[1]].tolist())
    ok, nd = _ulp_close(dgu[:, 128], ur.grad)
    assert ok, ("dswiglu up", nd, xs[nd[1]].tolist(), other[nd[1]].tolist())


@pytest.mark.parametrize("V,rows,skip,bad", [(4, 8192, -1, False), (50304, 180992, 50303, False),
                                             (128264, 1087 * 3, 128256, False), (1, 300, -1, False),
                                             (1000, 5000, 7, True), (50304, 700, 50303, False),
                                             (2, 180992, -1, False),  # 90k rows per id
                                             (128264, 256 * 1087, 128256, False)])
def test_embed_segments_device_matches_host_sort(K, V, rows, skip, bad):
    """mmpt_embed_segments (device counting sort + segment build) gives exactly the host
    restatement's order (engine.sort_segments: stable numpy argsort): seg_id, seg_off and
    perm bitwise, the count left in device memory; image-slot ids (skip) and out-of-range
    ids are excluded, the latter raise the device `bad` flag."""
    import numpy as np

    from multimodal_llm_pretraining_amd.engine import sort_segments

    torch.manual_seed(12)
    ids = torch.randint(0, V, (rows,), device=dev)
    if skip >= 0:
        ids[torch.rand(rows, device=dev) < 0.3] = skip
    if bad:
        ids[17], ids[rows - 1] = V + 5, -3
    seg_id, seg_off, perm, nseg, badf = K.embed_segments(ids, V, skip)
    idn = ids.cpu().numpy()
    keep = (idn != skip) & (idn >= 0) & (idn < V)
    r_id, r_off, r_perm = sort_segments(idn, np.flatnonzero(keep))
    n = int(nseg.item())
    assert n == r_id.size
    assert np.array_equal(seg_id[:n].cpu().numpy(), r_id)
    assert np.array_equal(seg_off[:n + 1].cpu().numpy(), r_off)
    assert np.array_equal(perm[:keep.sum()].cpu().numpy(), r_perm)
    assert int(badf.item()) == int(bad)


@pytest.mark.parametrize("V,pad", [(50304, 1), (128264, 128002)])
def test_embed_segments_linear_with_one_dominant_id(K, V, pad):
    """the reference's collators pad with one id (src/data/llava_data.py:95,
    scienceqa.py:83), so one id can cover most rows of a micro-batch.  The radix-sorted order
    is exact there too and costs what a uniform batch costs (round 4's rank step was
    quadratic in that id's count): 256 x 707 rows, 95% of them one id."""
    import time

    import numpy as np

    from multimodal_llm_pretraining_amd.engine import sort_segments

    rows = 256 * 707
    torch.manual_seed(14)
    uni = torch.randint(0, V, (rows,), device=dev)
    ids = uni.clone()
    ids[torch.rand(rows, device=dev) < 0.95] = pad

    def timed(x):
        K.embed_segments(x, V, -1)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(5):
            out = K.embed_segments(x, V, -1)
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / 5, out

    t_uni, _ = timed(uni)
    t_pad, (seg_id, seg_off, perm, nseg, _) = timed(ids)
    idn = ids.cpu().numpy()
    r_id, r_off, r_perm = sort_segments(idn, np.arange(rows))
    n = int(nseg.item())
    assert n == r_id.size
    assert np.array_equal(seg_id[:n].cpu().numpy(), r_id)
    assert np.array_equal(seg_off[:n + 1].cpu().numpy(), r_off)
    assert np.array_equal(perm.cpu().numpy(), r_perm)
    assert t_pad < 3 * t_uni + 2e-4, (t_pad, t_uni)


@pytest.mark.parametrize("V,pad", [(50304, 1), (128264, 128002)])
def test_embed_bwd_long_segment_split(K, V, pad):
    """a padded batch (one id on 95% of 256 x 707 rows, the reference collators'
    pad id, src/data/llava_data.py:95) — the long segment is summed over 256-row chunks of the
    sorted order and the chunk sums added in order (mmpt_embed_bwd_split): within fp32 rounding
    of the fp64 sum, deterministic, every short segment bitwise the serial kernel's, and the
    backward costs at most 3x the uniform-id batch's."""
    import time

    rows, h = 256 * 707, 2048
    torch.manual_seed(15)
    uni = torch.randint(0, V, (rows,), device=dev)
    ids = uni.clone()
    ids[torch.rand(rows, device=dev) < 0.95] = pad
    dout = torch.randn(rows, h, device=dev)
    base = torch.zeros(V, h, device=dev)

    def timed(x):
        seg = K.embed_segments(x, V, -1)
        t = base.clone()
        K.embed_bwd(seg, dout, t)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            K.embed_bwd(seg, dout, t)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / 5, seg

    t_uni, _ = timed(uni)
    t_pad, seg = timed(ids)
    print(f"embed_bwd 256x707: uniform {t_uni * 1e3:.3f} ms, 95% one id {t_pad * 1e3:.3f} ms")
    assert t_pad < 3 * t_uni + 2e-4, (t_pad, t_uni)
    got = base.clone()
    K.embed_bwd(seg, dout, got)
    again = base.clone()
    K.embed_bwd(seg, dout, again)
    assert torch.equal(got, again)  # deterministic
    # the long segment against fp64
    m = ids == pad
    ref = dout[m].double().sum(0)
    n = int(m.sum())
    assert (got[pad].double() - ref).abs().max().item() < 4 * n * 2.0 ** -24 * dout[m].abs().max().item()
    # short segments: bitwise the serial kernel (host segments, mmpt_embed_bwd)
    serial = base.clone()
    K.embed_bwd(_segments(ids), dout, serial)
    keep = torch.ones(V, dtype=torch.bool, device=dev)
    keep[pad] = False
    assert torch.equal(got[keep], serial[keep])


def test_embed_bwd_device_segments_bitwise(K):
    """The grid-stride embedding backward over device segments equals the host-segment
    kernel bitwise (same position-ordered fp32 sums, one writer per table row)."""
    torch.manual_seed(13)
    V, rows, h = 50304, 45248, 2048
    ids = torch.randint(0, 300, (rows,), device=dev)  # heavy collisions
    dout = torch.randn(rows, h, device=dev)
    base = torch.randn(V, h, device=dev)
    a, b = base.clone(), base.clone()
    K.embed_bwd(_segments(ids), dout, a)
    K.embed_bwd(K.embed_segments(ids, V, -1), dout, b)
    assert torch.equal(a, b)


@pytest.mark.parametrize("name,text_len", [("tiny-mm", 47), ("tiny-lm", 130)])
def test_batch_staged_from_host_on_copy_stream(K, name, text_len):
    """engine.Batch built from pinned host tensors on a copy stream (the bench's per-step
    staging: no device sync, device id sort) and from device tensors (the drop-in module's
    path) give the same bookkeeping and bit-identical loss and gradients."""
    from multimodal_llm_pretraining_amd import config as C
    from multimodal_llm_pretraining_amd.engine import Batch, Engine
    from multimodal_llm_pretraining_amd.params import ParamStore, init_normal
    from test_parity_gpu import oracle_cfg

    from oracle import model as O

    cfg = C.get_config(name)
    batch = O.make_batch(oracle_cfg(cfg), 3, text_len, seed=4)
    store = ParamStore(C.param_shapes(cfg), "cuda")
    init_normal(store, 0, cfg=cfg)
    eng = Engine(cfg, store)
    copy = torch.cuda.Stream()
    pinned = {k: v.pin_memory() for k, v in batch.items()}
    bh = Batch(cfg, pinned["input_ids"], pinned["labels"], pinned.get("pixel_values"), store.device,
               stream=copy)
    dv = {k: v.to(dev) for k, v in batch.items()}
    bd = Batch(cfg, dv["input_ids"], dv["labels"], dv.get("pixel_values"), store.device)
    assert bh.num_items == bd.num_items
    results = []
    for b in (bh, bd):
        store.zero_grad()
        loss = eng.forward(b, 1.0 / b.num_items)
        eng.backward(b)
        results.append((loss.clone(), store.grad.clone()))
    for t in ("ids", "labels", "loss_rows", "loss_labels", "loss_map", "img_map", "pixels"):
        x, y = getattr(bh, t), getattr(bd, t)
        assert (x is None) == (y is None) and (x is None or torch.equal(x, y)), t
    assert torch.equal(results[0][0], results[1][0])
    assert torch.equal(results[0][1], results[1][1])


def test_transpose_batched_matches_per_weight(K):
    """ParamStore.refresh_transposed: every W^T in one launch (mmpt_transpose_bf16_batched,
    ABI 14) — partial 64-tiles, a 1-D parameter between the weights, a subset of the names —
    bit for bit the transposes."""
    from multimodal_llm_pretraining_amd.params import ParamStore

    shapes = {"a": (200, 72), "bias": (768,), "b": (64, 64), "c": (3072, 768), "d": (8, 4104)}
    st = ParamStore(shapes, dev, grads=False)
    st.transposed = ["a", "b", "c", "d"]
    torch.manual_seed(5)
    st.shadow.copy_(torch.randn(st.padded, device=dev).to(torch.bfloat16))
    st.shadow_t.fill_(float("nan"))
    st.refresh_transposed()
    for n in st.transposed:
        assert torch.equal(st.wt(n), st.w(n).t()), n
    st.shadow_t.fill_(float("nan"))
    st.refresh_transposed(["c", "a"])
    assert torch.equal(st.wt("c"), st.w("c").t()) and torch.equal(st.wt("a"), st.w("a").t())
    assert torch.isnan(st.wt("b").float()).all()  # not in the list: untouched
