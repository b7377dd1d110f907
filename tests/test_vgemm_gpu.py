"""The ViT trunk's large bf16 GEMMs (``k_vgemm.hip``, the ``dfd_vgemm`` seam) against plain-PyTorch
fp32 products of the same bf16 operands (the C5 config's linears, ``src/models.py:88-107`` via timm
``vit_base_patch16_224``: qkv / proj / fc1 / fc2 forward, their data gradients and weight gradients).

Bounds: NT outputs are bf16, so each element is compared with the fp32 reference rounded to bf16
within 2 bf16 ulps (rtol 8e-3) plus an absolute term of 1e-3 x the reference's RMS (fp32 summation
order); the GELU epilogue (G = gelu, C = gelu' of the rounded pre-activation) within 2 ulps + 2e-3
(a pre-activation one rounding step away moves gelu' by up to ~1e-3); TN weight gradients are fp32: relative L2 error <= 1e-5.  Shapes cover ragged row counts
(M not a multiple of the 256-row tile, and for TN not a multiple of the 64-row m-step, whose rows
past the end must contribute zero), every epilogue, and the C5 token-row count at 8 images."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from deepfake_amd import _lib

pytestmark = pytest.mark.gpu

P = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731


def _nt(cuda, M, N, K, epi, seed, op=0):
    g = torch.Generator(device=cuda).manual_seed(seed)
    A = torch.randn(M, K, device=cuda, generator=g).bfloat16()
    B = (torch.randn(N, K, device=cuda, generator=g) / K ** 0.5).bfloat16()
    bias = torch.randn(N, device=cuda, generator=g) if epi & 1 else None
    R = torch.randn(M, N, device=cuda, generator=g).bfloat16() if epi & 2 else None
    Z = torch.randn(M, N, device=cuda, generator=g).bfloat16() if epi & 8 else None
    G = torch.full((M, N), float("nan"), device=cuda, dtype=torch.bfloat16) if epi & 4 else None
    C = torch.full((M, N), float("nan"), device=cuda, dtype=torch.bfloat16)
    lib = _lib.load()
    _lib.check(lib.dfd_vgemm(None, op, P(A), P(B), P(C), P(R), P(bias), P(Z), P(G), M, N, K, epi, None, 0))
    torch.cuda.synchronize()
    ref = A.float() @ B.float().T
    if bias is not None:
        ref = ref + bias
    if R is not None:
        ref = ref + R.float()
    if Z is not None:  # VG_DGELU: Z holds the derivative a VG_GELU2 forward stored
        ref = ref * Z.float()
    return C, G, ref


def _gelu_pair(pre):
    """gelu and gelu' (exact erf) of the bf16-rounded pre-activation"""
    z = pre.bfloat16().float().requires_grad_(True)
    g = F.gelu(z)
    return g.detach(), torch.autograd.grad(g.sum(), z)[0]


def _close(got, ref):
    scale = float(ref.float().pow(2).mean().sqrt())
    torch.testing.assert_close(got.float(), ref.bfloat16().float(), rtol=8e-3, atol=1e-3 * scale)


@pytest.mark.parametrize("op", [4, 5])  # 256- / 128-wide tiles (op 0 picks one by shape)
@pytest.mark.parametrize("M,N,K,epi", [(600, 256, 64, 0), (394, 768, 768, 1), (394, 2304, 768, 1),
                                       (1000, 768, 3072, 3), (394, 3072, 768, 5), (777, 3072, 768, 8),
                                       (8 * 197, 768, 2304, 0)])
def test_vgemm_nt_vs_fp32(cuda, M, N, K, epi, op):
    C, G, ref = _nt(cuda, M, N, K, epi, M + N + K + epi, op)
    if G is None:
        _close(C, ref)
    else:  # VG_GELU2: G = gelu(pre), C = gelu'(pre) of the rounded pre-activation
        g, d = _gelu_pair(ref)
        torch.testing.assert_close(G.float(), g.bfloat16().float(), rtol=8e-3, atol=2e-3)
        torch.testing.assert_close(C.float(), d.bfloat16().float(), rtol=8e-3, atol=2e-3)


def _tn_slab(lib, M, N, K, op, cuda):
    """op 1's slab; op 6 also carves its tile counters from the slab's end"""
    extra = 2 * (N // 256) * (K // 256) + 64 if op == 6 else 0
    return torch.empty(lib.dfd_vgemm_tn_slab_floats(M, N, K) + extra, device=cuda)


@pytest.mark.parametrize("op", [1, 6])  # 6: the splits reduced inside the launch (cooperative)
@pytest.mark.parametrize("colsum", [False, True, "adjacent"])
@pytest.mark.parametrize("M,N,K", [(394, 768, 256), (8 * 197, 768, 3072), (100, 256, 512), (4096, 2304, 768)])
def test_vgemm_tn_vs_fp32(cuda, M, N, K, colsum, op):
    """weight gradient; with colsum the bias gradient (column sums of A) from the same launch, rows past
    the end of the last m-step contributing zero ("adjacent": the bias gradient stored right after the
    weight gradient, as in the flat gradient buffer, reduced in one pass)"""
    g = torch.Generator(device=cuda).manual_seed(M * 7 + N)
    A = torch.randn(M, N, device=cuda, generator=g).bfloat16()
    B = torch.randn(M, K, device=cuda, generator=g).bfloat16()
    lib = _lib.load()
    slab = _tn_slab(lib, M, N, K, op, cuda)
    if colsum == "adjacent":
        flat = torch.full((N * K + N,), float("nan"), device=cuda)
        W, cs = flat[:N * K].view(N, K), flat[N * K:]
    else:
        W = torch.full((N, K), float("nan"), device=cuda)
        cs = torch.full((N,), float("nan"), device=cuda) if colsum else None
    _lib.check(lib.dfd_vgemm(None, op, P(A), P(B), P(W), None, None, None, P(cs), M, N, K, 0, P(slab), slab.numel()))
    torch.cuda.synchronize()
    ref = A.double().T @ B.double()
    e = float((W.double() - ref).norm() / ref.norm())
    assert e <= 1e-5, e
    if colsum:
        rc = A.double().sum(0)
        ec = float((cs.double() - rc).norm() / rc.norm())
        assert ec <= 1e-5, ec


C5_M = 128 * 197  # the ViT line's token rows (128 images x 197 tokens)


@pytest.mark.parametrize("N,K", [(2304, 768), (768, 768), (3072, 768), (768, 3072), (768, 2304)])
def test_vgemm_nt_c5_rows(cuda, N, K):
    """the ViT-B/16 linears and data gradients (qkv / proj / fc1 / fc2 forward, fc2 / qkv data gradients)
    at the C5 line's own M = 25,216: the tile width (256 vs 128 columns) and the dispatch-wave count
    follow M (vgemm_nt_bn), so the configuration the 128-image step runs is checked here, not only at
    <= 8 images"""
    C, _, ref = _nt(cuda, C5_M, N, K, 1, N + K)
    _close(C, ref)


@pytest.mark.parametrize("op", [1, 6])
@pytest.mark.parametrize("N,K", [(2304, 768), (768, 768), (3072, 768), (768, 3072)])
def test_vgemm_tn_c5_rows(cuda, N, K, op):
    """the four ViT weight gradients (dW = dY^T X, with the bias gradient from the same launch) at the
    C5 M = 25,216, where vgemm_tn_splits picks its split count and slab layout from M (e.g. 28 splits
    for 768 x 768 against 16 at M = 4,096): fp32 result against fp64, relative L2 <= 1e-5"""
    g = torch.Generator(device=cuda).manual_seed(N * 3 + K)
    A = torch.randn(C5_M, N, device=cuda, generator=g).bfloat16()
    B = torch.randn(C5_M, K, device=cuda, generator=g).bfloat16()
    lib = _lib.load()
    slab = _tn_slab(lib, C5_M, N, K, op, cuda)
    flat = torch.full((N * K + N,), float("nan"), device=cuda)
    W, cs = flat[:N * K].view(N, K), flat[N * K:]
    _lib.check(lib.dfd_vgemm(None, op, P(A), P(B), P(W), None, None, None, P(cs), C5_M, N, K, 0, P(slab), slab.numel()))
    torch.cuda.synchronize()
    ref = A.double().T @ B.double()
    e = float((W.double() - ref).norm() / ref.norm())
    rc = A.double().sum(0)
    ec = float((cs.double() - rc).norm() / rc.norm())
    print(f"TN op {op} {N}x{K} at M={C5_M}: slab splits {slab.numel() // (N * K + N)}, rel err {e:.2e}, bias {ec:.2e}")
    assert e <= 1e-5 and ec <= 1e-5, (e, ec)


@pytest.mark.parametrize("op,M", [(1, 2 * 197), (6, 2 * 197), (6, C5_M)])
def test_vgemm_deterministic(cuda, op, M):
    """runs of the same TN product are bit-identical (fixed-order slab sums; op 6: each split sums its
    rows over the splits in split order whatever the arrival order at the tile barrier), also across
    back-to-back launches that reuse the same counters (zero at rest)"""
    N, K = 768, 768
    A = torch.randn(M, N, device=cuda).bfloat16()
    B = torch.randn(M, K, device=cuda).bfloat16()
    lib = _lib.load()
    slab = _tn_slab(lib, M, N, K, op, cuda)
    outs = []
    for _ in range(3):
        W = torch.empty(N, K, device=cuda)
        _lib.check(lib.dfd_vgemm(None, op, P(A), P(B), P(W), None, None, None, None, M, N, K, 0, P(slab), slab.numel()))
        outs.append(W)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


def test_vgemm_refuses_uncovered(cuda):
    A = torch.zeros(64, 128, device=cuda).bfloat16()
    B = torch.zeros(200, 128, device=cuda).bfloat16()
    C = torch.zeros(64, 200, device=cuda).bfloat16()
    lib = _lib.load()
    assert lib.dfd_vgemm(None, 0, P(A), P(B), P(C), None, None, None, None, 64, 200, 100, 0, None, 0) != 0  # K % 64
    assert lib.dfd_vgemm(None, 0, P(A), P(B), P(C), None, None, None, None, 64, 200, 128, 0, None, 0) != 0  # N % 64


def test_vgemm_nt_tile_widths_agree(cuda):
    """the two tile widths sum every output's K in the same order: bit-identical results (and op 0's
    shape rule picks one of them), 128-wide-only N (N % 256 != 0) refused by the 256-wide op"""
    outs = [_nt(cuda, 1000, 768, 768, 3, 5, op)[0] for op in (0, 4, 5)]
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[1], outs[2])
    C, _, ref = _nt(cuda, 300, 640, 128, 1, 9, 0)  # N = 5 x 128
    _close(C, ref)
    A = torch.zeros(64, 128, device=cuda).bfloat16()
    B = torch.zeros(640, 128, device=cuda).bfloat16()
    C = torch.zeros(64, 640, device=cuda).bfloat16()
    assert _lib.load().dfd_vgemm(None, 4, P(A), P(B), P(C), None, None, None, None, 64, 640, 128, 0, None, 0) != 0


@pytest.mark.parametrize("M,N,K,epi", [(1000, 768, 768, 3), (394, 3072, 768, 5), (777, 3072, 768, 8),
                                       (300, 2304, 64, 1), (8 * 197, 768, 2304, 0)])
def test_vgemm_nt_xp_bit_identical(cuda, M, N, K, epi):
    """the fragment-pipelined K loop (knob vg_xp, through the dfd_set_tuning seam) issues the same
    MFMAs in the same order per output: bit-identical to the default loop at both tile widths,
    one-K-step products (K = 64) included"""
    lib = _lib.load()
    outs = {}
    prev = None
    try:
        for xp in (3, 0):
            p = lib.dfd_set_tuning(b"vg_xp", xp)
            prev = p if prev is None else prev
            outs[xp] = [_nt(cuda, M, N, K, epi, 17, op)[:2] for op in (4, 5) if N % 256 == 0 or op == 5]
    finally:
        if prev is not None:  # the seam's previous value (the default loop unless a test changed it)
            lib.dfd_set_tuning(b"vg_xp", prev)
    for (c3, g3), (c0, g0) in zip(outs[3], outs[0]):
        assert torch.equal(c3, c0)
        assert (g3 is None) == (g0 is None) and (g3 is None or torch.equal(g3, g0))


@pytest.mark.parametrize("M,K,epi", [(1000, 64, 19), (777, 256, 17), (300, 576, 1), (64, 64, 3)])
def test_vgemm_nt_64_wide(cuda, M, K, epi):
    """the 64-wide tile (N % 128 != 0: ResNet-50 layer1's Cout 64) with the bias / identity / ReLU
    epilogues, against the fp32 product"""
    C, _, ref = _nt(cuda, M, 64, K, epi & 3, M + K + epi, 0)
    if epi & 16:  # VG_RELU: rerun with ReLU (the helper's reference has none)
        g = torch.Generator(device=cuda).manual_seed(M + K + epi)
        A = torch.randn(M, K, device=cuda, generator=g).bfloat16()
        B = (torch.randn(64, K, device=cuda, generator=g) / K ** 0.5).bfloat16()
        bias = torch.randn(64, device=cuda, generator=g)
        R = torch.randn(M, 64, device=cuda, generator=g).bfloat16() if epi & 2 else None
        C = torch.full((M, 64), float("nan"), device=cuda, dtype=torch.bfloat16)
        _lib.check(_lib.load().dfd_vgemm(None, 0, P(A), P(B), P(C), P(R), P(bias), None, None, M, 64, K, epi, None, 0))
        torch.cuda.synchronize()
        ref = A.float() @ B.float().T + bias
        if R is not None:
            ref = ref + R.float()
        ref = torch.relu(ref)
    _close(C, ref)
