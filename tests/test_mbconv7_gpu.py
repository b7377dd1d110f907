"""The fused 7x7-stage MBConv forward (``k_mbconv7.hip``: blocks.5.1-5.3 and 6.0, one workgroup per
frame, grid-wide barriers for the training-mode BatchNorm statistics) against the plan's unfused
launches (expansion GEMM -> BN1 finalize -> depthwise -> BN2 finalize -> SE squeeze/excite ->
projection GEMM -> BN3 finalize -> BN apply) on the same bf16 inputs and weights.

Both paths round every stored tensor to bf16 at the same points and sum the per-channel BatchNorm
statistics in fp32 per frame then double over frames; only the summation order inside a frame
differs, so a saved tensor may differ by one bf16 ulp in a few elements.  Bounds: relative L2 error
of every saved activation <= ``SAVED_TOL`` (a 1-ulp flip in every element would be 2^-8 = 3.9e-3),
BN buffers rtol 1e-4, features rtol 2e-2 (bf16 end to end), gradients cosine >= 0.9995.
The end-to-end bf16 parity against the fp32 oracle runs through the fused path by default
(``test_b0_bench_config_gpu.py``, ``test_b0_224_gpu.py``)."""
import ctypes

import pytest
import torch

from deepfake_amd import _lib
from deepfake_amd.pretrained_detector import PretrainedBackboneDetector
from deepfake_amd.weights import deterministic_init_

pytestmark = pytest.mark.gpu

HW = 224
SEED = 41
SAVED_TOL = 4e-3


def _frames(n, cuda):
    g = torch.Generator().manual_seed(n)
    return torch.randint(0, 256, (n, 3, HW, HW), generator=g, dtype=torch.uint8).to(cuda)


def _model(cuda, fused, training=True):
    det = PretrainedBackboneDetector("efficientnet_b0", pretrained=False, num_classes=2, dropout_rate=0.0,
                                     compute_dtype="bf16")
    deterministic_init_(det, seed=SEED)
    det = det.to(cuda).train(training)
    det.ensure_flat()
    rt = det.backbone.runtime()
    rt.set_input_norm("imagenet")
    rt.set_tuning("mbconv7", 1 if fused else 0)
    return det, rt


def _saved(lib, h, ws):
    off, rows, cols = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    out, i = [], 0
    while lib.dfd_b0_saved_tensor(h, i, ctypes.byref(off), ctypes.byref(rows), ctypes.byref(cols)) == 0:
        n = rows.value * cols.value
        out.append(ws[off.value:off.value + 2 * n].view(torch.bfloat16).view(rows.value, cols.value).float().clone())
        i += 1
    return out


def _fused_info(lib, h, ws):
    nb, off = ctypes.c_int(), ctypes.c_int64()
    _lib.check(lib.dfd_b0_fused_info(h, ctypes.byref(nb), ctypes.byref(off)))
    abort = int(ws[off.value:off.value + 4].view(torch.int32).item())
    return nb.value, abort


def _forward(cuda, fused, frames, training=True):
    lib = _lib.load()
    det, rt = _model(cuda, fused, training)
    x = _frames(frames, cuda)
    with torch.no_grad():
        feats, (h, ws) = rt.forward(x, det, 1, training)
        torch.cuda.synchronize()
        saved = _saved(lib, h, ws) if training else []
        nb, abort = _fused_info(lib, h, ws)
    bufs = {n: b.detach().clone() for n, b in det.named_buffers() if "running" in n}
    return dict(feats=feats.float().clone(), saved=saved, nb=nb, abort=abort, bufs=bufs, det=det, rt=rt, h=h, ws=ws,
                x=x)


def _rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.parametrize("frames", [256, 96])
def test_fused_training_forward_matches_unfused(cuda, frames):
    ref = _forward(cuda, False, frames)
    got = _forward(cuda, True, frames)
    assert ref["nb"] == 0
    assert got["nb"] == 4, "blocks.5.1-5.3 and 6.0 take the fused path at 7x7"
    assert got["abort"] == 0, "grid barrier abort: the fused grid was not co-resident"
    assert len(got["saved"]) == len(ref["saved"])
    errs = [_rel(g, r) for g, r in zip(got["saved"], ref["saved"])]
    worst = max(range(len(errs)), key=lambda i: errs[i])
    print(f"{frames} frames: worst saved-tensor rel err {errs[worst]:.2e} (saved #{worst} of {len(errs)})")
    assert errs[worst] <= SAVED_TOL, (worst, errs[worst])
    for n, rb in ref["bufs"].items():
        torch.testing.assert_close(got["bufs"][n], rb, rtol=1e-4, atol=1e-6, msg=lambda m: f"{n}: {m}")
    torch.testing.assert_close(got["feats"], ref["feats"], rtol=2e-2, atol=2e-2)
    assert _rel(got["feats"], ref["feats"]) <= SAVED_TOL


def test_fused_eval_forward_matches_unfused(cuda):
    ref = _forward(cuda, False, 64, training=False)
    got = _forward(cuda, True, 64, training=False)
    assert got["nb"] == 4
    err = _rel(got["feats"], ref["feats"])
    print(f"eval features rel err {err:.2e}")
    assert err <= SAVED_TOL


def test_fused_training_step_gradients(cuda):
    """Full trunk backward after the fused forward: the backward reads the fused kernel's saved
    tensors and BN buffers exactly as it reads the unfused launches' ones."""
    out = {}
    for fused in (False, True):
        r = _forward(cuda, fused, 128)
        g = torch.Generator(device=cuda).manual_seed(3)
        dfeat = torch.randn(128, 1280, device=cuda, generator=g) * 1e-3
        grads = torch.zeros_like(r["det"]._flat_p)
        with torch.no_grad():
            r["rt"].backward(r["h"], r["ws"], r["x"], dfeat, r["det"], grads, True, 0, 9)
        torch.cuda.synchronize()
        po = r["det"].param_offsets()
        out[fused] = {n: grads[po[n]:po[n] + p.numel()].double().clone() for n, p in r["det"].named_parameters()}
    scale = max(float(v.norm()) for v in out[False].values())
    bad = []
    for n, rg in out[False].items():
        gg = out[True][n]
        rn = float(rg.norm())
        if rn <= 1e-3 * scale:
            continue  # structurally ~zero (bn3 biases): rounding residue on both sides
        cos = float(gg @ rg) / (float(gg.norm()) * rn + 1e-30)
        if cos < 0.9995 or abs(float(gg.norm()) - rn) > 1e-2 * rn:
            bad.append((n, round(cos, 6), round(float(gg.norm()) / rn, 5)))
    print(f"fused vs unfused gradients: {len(out[False])} tensors, outside {bad}")
    assert not bad


def test_fused_skipped_for_fp32(cuda):
    lib = _lib.load()
    det = PretrainedBackboneDetector("efficientnet_b0", pretrained=False, num_classes=2, dropout_rate=0.0,
                                     compute_dtype="fp32")
    deterministic_init_(det, seed=SEED)
    det = det.to(cuda).train()
    det.ensure_flat()
    rt = det.backbone.runtime()
    with torch.no_grad():
        _, (h, ws) = rt.forward(_frames(8, cuda), det, 0, True)
    nb, _ = _fused_info(lib, h, ws)
    assert nb == 0
