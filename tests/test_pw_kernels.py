"""1x1-conv kernels (dfd_pw_conv / dfd_pw_conv_wgrad) against a plain PyTorch fp32 reference.

The trunk's conv_pw / conv_pwl / conv_head run as C[M][N] = pro(A)[M][K] . W[N][K]^T on NHWC
rows, where pro() is the producing layer's BatchNorm+SiLU (+ squeeze-excite gate), replacing
aten conv2d(kernel_size=1) inside timm's MBConv blocks (reached from
src/pretrained_detector.py:116).  bf16 storage: the reference takes the same bf16-rounded
operands (the kernel rounds pro(A) to bf16 before the MFMA) and accumulates in fp32; the output
is bf16-rounded, so it is compared at bf16 resolution.  Both the streaming kernel (tall layers)
and the tiled kernel (everything else) are exercised via dfd_set_tuning("stream_min_rows").
"""
import ctypes

import pytest
import torch

from deepfake_amd import _lib

pytestmark = pytest.mark.gpu


def _lib_():
    return _lib.load()


def _pro(a, mode, scale, shift, gate, rpf):
    x = a.float()
    if mode == 0:
        return x
    if mode == 4:  # already-activated input times the SE gate
        f = torch.arange(x.shape[0], device=x.device) // rpf
        return x * gate[f]
    x = torch.nn.functional.silu(x * scale + shift)
    if mode == 2:
        f = torch.arange(x.shape[0], device=x.device) // rpf
        x = x * gate[f]
    return x


TDT = {1: torch.bfloat16, 2: torch.float16}  # DFD_DTYPE_BF16 / DFD_DTYPE_F16 storage


def _inputs(M, N, K, mode, rpf, seed, dev, dt=1):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    a = torch.randn(M, K, generator=g, device=dev).to(TDT[dt])
    w = (torch.randn(N, K, generator=g, device=dev) / K ** 0.5).to(TDT[dt])
    scale = torch.rand(K, generator=g, device=dev) + 0.5
    shift = torch.randn(K, generator=g, device=dev) * 0.1
    frames = (M + rpf - 1) // rpf
    gate = torch.rand(frames, K, generator=g, device=dev)
    return a, w, scale, shift, gate


def _run(M, N, K, mode, resid, stats, stream_min_rows, dev, rpf=3136, seed=0, tile=-1, sk=0, dt=1):
    lib = _lib_()
    a, w, scale, shift, gate = _inputs(M, N, K, mode, rpf, seed, dev, dt)
    gr = torch.Generator(device=dev)
    gr.manual_seed(seed + 1)
    r = torch.randn(M, N, generator=gr, device=dev).to(TDT[dt]) if resid else None
    c = torch.empty(M, N, device=dev, dtype=TDT[dt])
    st = torch.zeros(1024 * 2 * N, device=dev) if stats else None
    rows = ctypes.c_int(0)
    prev = lib.dfd_set_tuning(b"stream_min_rows", stream_min_rows)
    prev_tile = lib.dfd_set_tuning(b"gemm_tile", tile)
    prev_sk = lib.dfd_set_tuning(b"pw_sk", sk)
    try:
        _lib.check(lib.dfd_pw_conv(_lib.stream_of(dev), dt, a.data_ptr(), w.data_ptr(), c.data_ptr(), _lib.ptr(r), M,
                                   N, K, mode, scale.data_ptr(), shift.data_ptr(), gate.data_ptr(), rpf,
                                   _lib.ptr(st), ctypes.byref(rows)))
        torch.cuda.synchronize()
    finally:
        lib.dfd_set_tuning(b"stream_min_rows", prev)
        lib.dfd_set_tuning(b"gemm_tile", prev_tile)
        lib.dfd_set_tuning(b"pw_sk", prev_sk)
    ap = _pro(a, mode, scale, shift, gate, rpf).to(TDT[dt]).float()
    ref = ap @ w.float().t()
    mag = ref.abs()
    if resid:
        # the kernel adds the residual to the fp32 accumulator and rounds once; a bf16 framework
        # rounds the conv output first, so near-cancelling sums may differ by one ulp of |conv|
        mag = mag + r.float().abs()
        ref = ref.to(TDT[dt]).float() + r.float()
    got = c.float()
    err = (got - ref).abs()
    tol = (1e-2 if dt == 1 else 2e-3) * (mag + ref.abs().mean())
    assert bool((err <= tol).all()), f"max err {float(err.max())} (ref mean {float(ref.abs().mean())})"
    if stats:
        n = rows.value
        assert 1 <= n <= 1024
        s = st.view(-1)[: n * 2 * N].view(n, 2, N).double().sum(0)
        torch.testing.assert_close(s[0], got.double().sum(0), rtol=1e-4, atol=1e-2)
        torch.testing.assert_close(s[1], (got.double() ** 2).sum(0), rtol=1e-4, atol=1e-2)


# (M, N, K, mode, resid, stats): the B0 1x1 shapes of the high-resolution stages, ragged M
STREAM_CASES = [
    (100355, 96, 16, 0, False, True),    # blocks.1.0 conv_pw
    (50021, 144, 24, 0, False, True),    # blocks.1.1 conv_pw (two N chunks)
    (20007, 240, 40, 0, False, True),    # blocks.2.1 conv_pw
    (20007, 480, 80, 0, False, True),    # blocks.3.x conv_pw
    (9999, 672, 112, 0, False, True),    # blocks.4.x conv_pw
    (100355, 16, 32, 2, False, True),    # blocks.0.0 conv_pw (project, gated)
    (50021, 24, 96, 2, False, True),     # blocks.1.0 conv_pwl
    (50021, 24, 144, 2, False, True),    # blocks.1.1 conv_pwl
    (20007, 40, 144, 2, False, True),    # blocks.2.0 conv_pwl
    (100355, 16, 96, 0, False, False),   # blocks.1.0 conv_pw dgrad
    (50021, 24, 144, 0, True, False),    # blocks.1.1 conv_pw dgrad + skip
    (20007, 40, 240, 0, True, False),    # blocks.2.1 conv_pw dgrad + skip
    (20007, 40, 240, 0, False, False),   # blocks.3.0 conv_pw dgrad
    (100355, 32, 16, 0, False, False),   # blocks.0.0 conv_pw dgrad
    (50021, 96, 24, 0, False, False),    # blocks.1.0 conv_pwl dgrad
    (50021, 144, 40, 0, False, False),   # blocks.2.0 conv_pwl dgrad
    (20007, 240, 40, 0, False, False),   # blocks.2.1 conv_pwl dgrad
    (20007, 480, 80, 0, False, False),   # blocks.3.x conv_pwl dgrad
]


@pytest.mark.parametrize("case", STREAM_CASES, ids=lambda c: "x".join(map(str, c[:3])) + f"_m{c[3]}r{int(c[4])}")
@pytest.mark.parametrize("path", ["stream", "tiled", "tiled128x128", "tiled128x64", "tiled64x64", "tiled32x64"])
def test_pw_conv_bf16(cuda, case, path):
    M, N, K, mode, resid, stats = case
    tile = {"tiled128x128": 0, "tiled128x64": 1, "tiled64x64": 2, "tiled32x64": 3}.get(path, -1)
    _run(M, N, K, mode, resid, stats, 0 if path == "stream" else 1 << 60, cuda, rpf=784 if M < 30000 else 3136,
         tile=tile)


# the tiled GEMM's shapes (late stages, 14x14 / 7x7 maps), every tile configuration
@pytest.mark.parametrize("case", [(12544, 192, 1152, 2, False, True), (12544, 1152, 192, 0, False, True),
                                  (12544, 1280, 320, 0, False, True), (12544, 320, 1280, 0, False, False),
                                  (50176, 112, 672, 2, False, True), (50176, 80, 480, 0, True, False),
                                  (12544, 192, 1152, 4, False, True), (50176, 112, 672, 4, False, True),
                                  (3001, 200, 104, 1, False, True)])
@pytest.mark.parametrize("tile", [-1, 0, 1, 2, 3])
def test_pw_conv_bf16_late_layers(cuda, case, tile):
    M, N, K, mode, resid, stats = case
    _run(M, N, K, mode, resid, stats, 0, cuda, rpf=49, tile=tile)


# the small-K weight-panel kernel (k_pw_sk.hip; dispatched for K <= 192 only, K = 320 measured slower):
# every (K, panel width) instantiation the 14x14 / 7x7
# stages and conv_head use, with the BN-stat epilogue, plain, and with the residual; rows past the
# 64-row multiple fall back to the other kernels (last case)
SK_CASES = [(12544, 1152, 192, 0, False, True),   # blocks.5.x / 6.0 conv_pw forward (K 192, BN 128)
            (12544, 1152, 192, 0, False, False),  # blocks.5.x conv_pwl data gradient
            (12544, 1280, 320, 0, False, True),   # conv_head forward (K 320, BN 64)
            (12544, 1152, 320, 0, False, False),  # blocks.6.0 conv_pwl data gradient
            (50176, 480, 80, 0, False, True),     # blocks.3.x / 4.0 conv_pw forward (K 80 -> 96, BN 96)
            (50176, 480, 80, 0, False, False),    # blocks.3.x conv_pwl data gradient
            (50176, 672, 112, 0, False, True),    # blocks.4.x / 5.0 conv_pw forward (K 112 -> 128, BN 96)
            (50176, 672, 112, 0, True, False),    # residual epilogue
            (640, 512, 192, 0, False, True),      # BN 128 with more workgroups than tiles
            (12550, 1152, 192, 0, False, True)]   # ragged rows: not covered, the tiled kernel runs


@pytest.mark.parametrize("case", SK_CASES, ids=lambda c: "x".join(map(str, c[:3])) + f"_r{int(c[4])}s{int(c[5])}")
def test_pw_conv_small_k_panel(cuda, case):
    M, N, K, mode, resid, stats = case
    _run(M, N, K, mode, resid, stats, 1 << 60, cuda, rpf=49, sk=1)


def test_pw_conv_rejects_bad_args(cuda):
    lib = _lib_()
    rows = ctypes.c_int(0)
    assert lib.dfd_pw_conv(None, 7, None, None, None, None, 16, 8, 8, 0, None, None, None, 0, None,
                           ctypes.byref(rows)) == -1
    assert b"dtype" in lib.dfd_last_error()
    assert lib.dfd_pw_conv(None, 1, None, None, None, None, 16, 8, 8, 2, None, None, None, 0, None,
                           ctypes.byref(rows)) == -1


def _run_wgrad(M, N, K, mode, stream_min_rows, dev, rpf=3136, seed=1, accumulate=False, wg_pf=None, dt=1):
    """dW[N][K] = sum_m dY[m][n] * pro(X)[m][k] (conv_pw / conv_pwl weight gradient)."""
    lib = _lib_()
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    dy = torch.randn(M, N, generator=g, device=dev).to(TDT[dt])
    x, _, scale, shift, gate = _inputs(M, N, K, mode, rpf, seed + 1, dev, dt)
    dw = torch.randn(N, K, device=dev) if accumulate else torch.empty(N, K, device=dev)
    dw0 = dw.clone()
    slab = torch.empty(8 << 20, device=dev)
    prev = lib.dfd_set_tuning(b"stream_min_rows", stream_min_rows)
    prev_pf = lib.dfd_set_tuning(b"wg_pf", wg_pf) if wg_pf is not None else None
    try:
        _lib.check(lib.dfd_pw_conv_wgrad(_lib.stream_of(dev), dt, dy.data_ptr(), x.data_ptr(), M, N, K, mode,
                                         scale.data_ptr(), shift.data_ptr(), gate.data_ptr(), rpf, slab.data_ptr(),
                                         slab.numel(), dw.data_ptr(), 1 if accumulate else 0))
        torch.cuda.synchronize()
    finally:
        lib.dfd_set_tuning(b"stream_min_rows", prev)
        if prev_pf is not None:
            lib.dfd_set_tuning(b"wg_pf", prev_pf)
    xp = _pro(x, mode, scale, shift, gate, rpf).to(TDT[dt]).double()
    ref = dy.double().t() @ xp
    if accumulate:
        ref = ref + dw0.double()
    torch.testing.assert_close(dw.double(), ref, rtol=1e-4, atol=1e-4 * float(ref.abs().max()))


WGRAD_CASES = [
    (100355, 96, 16, 0),    # blocks.1.0 conv_pw
    (50021, 144, 24, 0),    # blocks.1.1 / 2.0 conv_pw
    (20007, 240, 40, 0),    # blocks.2.1 / 3.0 conv_pw
    (100355, 16, 32, 2),    # blocks.0.0 conv_pw (gated)
    (50021, 24, 96, 2),     # blocks.1.0 conv_pwl
    (50021, 24, 144, 2),    # blocks.1.1 conv_pwl
    (20007, 40, 144, 2),    # blocks.2.0 conv_pwl
    (20007, 40, 240, 2),    # blocks.2.1 conv_pwl
]


@pytest.mark.parametrize("case", WGRAD_CASES, ids=lambda c: "x".join(map(str, c)))
@pytest.mark.parametrize("path", ["stream", "tiled"])
def test_pw_conv_wgrad_bf16(cuda, case, path):
    M, N, K, mode = case
    _run_wgrad(M, N, K, mode, 0 if path == "stream" else 1 << 60, cuda, rpf=784 if M < 30000 else 3136)


@pytest.mark.parametrize("case", [(12544, 192, 1152, 4), (50176, 80, 480, 4), (3001, 40, 240, 4)],
                         ids=lambda c: "x".join(map(str, c)))
def test_pw_conv_wgrad_gate_bf16(cuda, case):
    """conv_pwl weight gradient on the materialised activation (mode 4: x * gate)."""
    M, N, K, mode = case
    _run_wgrad(M, N, K, mode, 0, cuda, rpf=49 if M < 20000 else 196)


def test_pw_conv_wgrad_accumulate(cuda):
    _run_wgrad(50021, 24, 96, 2, 0, cuda, accumulate=True)
    _run_wgrad(12544, 192, 1152, 2, 0, cuda, rpf=49, accumulate=True)


@pytest.mark.parametrize("case", [(12544, 1152, 192, 0), (50176, 672, 112, 0), (12544, 1152, 320, 0), (3001, 96, 40, 0),
                                  (12544, 1152, 192, 1), (777, 64, 48, 0)],
                         ids=lambda c: "x".join(map(str, c)))
@pytest.mark.parametrize("wg_pf", [1, 2])
def test_pw_conv_wgrad_tiled_ring(cuda, case, wg_pf):
    """the tiled weight gradient with one / two m-steps of loads in flight (knob wg_pf): the late-stage
    conv_pw shapes (12,544 / 50,176 rows), ragged row counts (the last ring slot of a split partly or
    wholly past the end) and a split shorter than the ring"""
    M, N, K, mode = case
    _run_wgrad(M, N, K, mode, 1 << 60, cuda, rpf=49, wg_pf=wg_pf)


# fp16 storage (DFD_DTYPE_F16, v_mfma_f32_16x16x32_f16): the generic 16-bit tile kernels (the streaming
# and weight-panel kernels are bf16-only); a forward / dgrad case of every prologue mode and tile, and
# the weight gradient of every prologue mode; tolerance scaled to fp16's 2^-11 rounding
@pytest.mark.parametrize("case", [STREAM_CASES[0], STREAM_CASES[5], STREAM_CASES[10], (12544, 192, 1152, 2, False, True),
                                  (12544, 1280, 320, 0, False, True), (50176, 112, 672, 4, False, True),
                                  (3001, 200, 104, 1, False, True)],
                         ids=lambda c: "x".join(map(str, c[:3])) + f"_m{c[3]}r{int(c[4])}")
@pytest.mark.parametrize("tile", [-1, 0, 2, 3])
def test_pw_conv_fp16(cuda, case, tile):
    M, N, K, mode, resid, stats = case
    _run(M, N, K, mode, resid, stats, 0, cuda, rpf=49 if M < 20000 else 3136, tile=tile, dt=2)


@pytest.mark.parametrize("case", [WGRAD_CASES[0], WGRAD_CASES[3], (12544, 192, 1152, 4), (12544, 1152, 192, 1),
                                  (777, 64, 48, 0)], ids=lambda c: "x".join(map(str, c)))
def test_pw_conv_wgrad_fp16(cuda, case):
    M, N, K, mode = case
    _run_wgrad(M, N, K, mode, 0, cuda, rpf=49 if M < 20000 else 3136, dt=2)
