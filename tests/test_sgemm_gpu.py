"""fp32 GEMM kernels of the recurrent models (k_rnn.hip): the large-tile MFMA kernel
(``sgemm_big_kernel``, 128 x 64 tiles, taken when M % 128 == N % 64 == K % 16 == 0) and the 64 x 64
kernel (every other shape), through the ``dfd_sgemm`` seam, against a float64 torch product of the
same operands.  fp32 products are exact on MFMA; only the summation order differs, so the bound is
|err| <= 1e-5 * (|A| |B|)[m][n] (the sum of the absolute products) elementwise."""
import ctypes

import pytest
import torch

from deepfake_amd import _lib

pytestmark = pytest.mark.gpu


def _run(cuda, ta, tb, M, N, K, beta, bias):
    g = torch.Generator(device=cuda).manual_seed(M * 7 + N * 3 + K + 2 * ta + tb)
    A = torch.randn((K, M) if ta else (M, K), device=cuda, generator=g)
    B = torch.randn((K, N) if tb else (N, K), device=cuda, generator=g)
    C = torch.randn(M, N, device=cuda, generator=g)
    bv = torch.randn(N, device=cuda, generator=g) if bias else None
    Am = A.t() if ta else A
    Bm = B if tb else B.t()
    ref = Am.double() @ Bm.double()
    mag = Am.double().abs() @ Bm.double().abs()
    if beta:
        ref = ref + beta * C.double()
        mag = mag + abs(beta) * C.double().abs()
    if bias:
        ref = ref + bv.double()
        mag = mag + bv.double().abs()
    lib = _lib.load()
    out = C.clone()
    _lib.check(lib.dfd_sgemm(None, int(ta), int(tb), ctypes.c_void_p(A.data_ptr()), A.shape[1],
                             ctypes.c_void_p(B.data_ptr()), B.shape[1], ctypes.c_void_p(out.data_ptr()), N, M, N, K,
                             float(beta), ctypes.c_void_p(bv.data_ptr()) if bias else None))
    torch.cuda.synchronize()
    err = (out.double() - ref).abs()
    assert bool((err <= 1e-5 * mag + 1e-6).all()), float((err / (mag + 1e-30)).max())


@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(256, 192, 1024), (3584, 512, 1024), (128, 64, 16), (100, 70, 33), (64, 512, 512)])
def test_sgemm_vs_float64(cuda, ta, tb, M, N, K):
    _run(cuda, ta, tb, M, N, K, 0.0, False)


@pytest.mark.parametrize("M,N,K", [(256, 128, 64), (96, 40, 24)])
def test_sgemm_beta_bias(cuda, M, N, K):
    _run(cuda, 0, 0, M, N, K, 1.0, True)
