"""CPU-side checks of the drop-in boundary (no GPU needed, no compute launched).

* the C-ABI library loads and exports every symbol ``include/dfd_hip.h`` declares, and the
  ctypes binding (``_lib._SIGS``) covers exactly that set;
* host-only entry points (tensor table, segment table) agree with the PyTorch module's
  ``state_dict`` layout, which itself matches the reference's keys and shapes
  (``pretrained_detector.py:42-49,65-76``);
* the module honours the reference's construction contract and refuses what it cannot do
  offline or without a HIP device (no silent CPU fallback).
"""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from deepfake_amd import _lib
from deepfake_amd.pretrained_detector import PretrainedBackboneDetector
from deepfake_amd.weights import deterministic_init_, hash_uniform
from oracle.detector_cpu import DetectorCPU

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "dfd_hip.h")


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"DFD_API\s+[\w\s\*]*?\b(dfd_\w+)\s*\(", src)))


def test_header_declares_expected_surface():
    names = _declared()
    assert "dfd_b0_forward" in names and "dfd_b0_backward" in names and "dfd_adam_step" in names
    assert len(names) >= 20


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_matches_header():
    assert sorted(_lib.EXPORTED) == _declared()


def test_exports_nothing_else():
    """-fvisibility=hidden: the only dynamic symbols with the dfd_ prefix are the ABI."""
    import subprocess

    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    syms = sorted({l.split()[-1] for l in out.splitlines() if l.split() and l.split()[-1].startswith("dfd_")})
    assert syms == _declared()


def test_host_entry_points():
    lib = _lib.load()
    assert lib.dfd_version() >= 1
    n = lib.dfd_b0_tensor_count()
    trunk = PretrainedBackboneDetector("efficientnet_b0", pretrained=False).backbone
    sd = trunk.state_dict()
    keys = list(sd.keys())  # timm state_dict order, counters included (DFD_TENSOR_COUNTER)
    assert n == len(keys) == 358
    name = ctypes.create_string_buffer(128)
    kind, ndim = ctypes.c_int(), ctypes.c_int()
    shape = (ctypes.c_int64 * 4)()
    for i in range(n):
        _lib.check(lib.dfd_b0_tensor_info(i, name, 128, ctypes.byref(kind), ctypes.byref(ndim), shape))
        k = name.value.decode()
        assert k == keys[i], (i, k, keys[i])
        assert tuple(shape[:ndim.value]) == tuple(sd[k].shape), k
        assert kind.value == (2 if k.endswith("num_batches_tracked") else 1 if "running" in k else 0), k
    # bad index -> error code + message, not a crash
    assert lib.dfd_b0_tensor_info(n, name, 128, ctypes.byref(kind), ctypes.byref(ndim), shape) != 0
    assert b"range" in lib.dfd_last_error()
    # backward segments tile the tensor table without gaps, head first
    nseg = lib.dfd_b0_segment_count()
    lo, hi = ctypes.c_int(), ctypes.c_int()
    spans = []
    for s in range(nseg):
        _lib.check(lib.dfd_b0_segment_tensors(s, ctypes.byref(lo), ctypes.byref(hi)))
        spans.append((lo.value, hi.value))
    assert spans[0][1] == n and spans[-1][0] == 0
    for a, b in zip(spans, spans[1:]):
        assert b[1] == a[0]


def test_state_dict_matches_reference_layout():
    det = PretrainedBackboneDetector("efficientnet_b0", pretrained=False, num_classes=2, dropout_rate=0.5)
    ref = DetectorCPU(num_classes=2, dropout_rate=0.5)
    a, b = det.state_dict(), ref.state_dict()
    assert list(a.keys()) == list(b.keys())
    for k in a:
        assert a[k].shape == b[k].shape and a[k].dtype == b[k].dtype, k
    assert sum(p.numel() for p in det.parameters()) == 4_418_047
    assert det.feature_dim == 1280 and det.backbone_name == "efficientnet_b0" and det.num_classes == 2


def test_state_dict_round_trip_through_flat_storage():
    ref = DetectorCPU()
    deterministic_init_(ref, seed=21)
    with torch.no_grad():
        for n, b in ref.named_buffers():
            if "running" in n:
                b.copy_(torch.from_numpy(hash_uniform(22, n, b.numel()).reshape(b.shape)).abs() + 0.5)
    det = PretrainedBackboneDetector("efficientnet_b0", pretrained=False)
    det.load_state_dict(ref.state_dict())
    det.ensure_flat()
    out = det.state_dict()
    for k, v in ref.state_dict().items():
        torch.testing.assert_close(out[k], v, rtol=0, atol=0)
    # parameters are views into one flat fp32 buffer (bucketed all-reduce / fused AdamW rely on it)
    flat = det._flat_p
    assert flat.numel() == 4_418_047
    for _, p in det.named_parameters():
        assert p.untyped_storage().data_ptr() == flat.untyped_storage().data_ptr()


def test_pretrained_true_refuses_offline():
    with pytest.raises(Exception):
        PretrainedBackboneDetector("efficientnet_b0", pretrained=True)


def test_unknown_backbone_raises():
    with pytest.raises(ValueError):
        PretrainedBackboneDetector("resnet18", pretrained=False)  # resnet50 is provided (inference)


def test_forward_on_cpu_raises_no_fallback():
    det = PretrainedBackboneDetector("efficientnet_b0", pretrained=False).eval()
    with pytest.raises(RuntimeError):
        det(torch.zeros(1, 2, 3, 64, 64))


def test_unfreeze_backbone_is_noop_for_b0():
    """pretrained_detector.py:95-101: `self.backbone` has no `.blocks` for EfficientNet (F8e)."""
    det = PretrainedBackboneDetector("efficientnet_b0", pretrained=False, freeze_backbone=True)
    before = [p.requires_grad for p in det.parameters()]
    det.unfreeze_backbone(3)
    assert [p.requires_grad for p in det.parameters()] == before


def test_hash_uniform_portable():
    a = hash_uniform(3, "x", 1000)
    assert a.dtype == np.float32 and a.min() >= -1.0 and a.max() < 1.0
    assert np.array_equal(a, hash_uniform(3, "x", 1000))
    assert not np.array_equal(a, hash_uniform(4, "x", 1000))


def test_train_step_auto_loss_scaling_sees_ensemble_members():
    """TrainStep(loss_scale="auto") turns dynamic loss scaling on when ANY submodule computes in fp16
    -- EnsembleDetector has no compute_dtype of its own -- and leaves it off otherwise."""
    from deepfake_amd.pretrained_detector import EnsembleDetector
    from deepfake_amd.trainer import TrainStep

    ens16 = EnsembleDetector(["efficientnet_b0", "efficientnet_b0"], pretrained=False, compute_dtype="fp16")
    assert TrainStep(ens16).loss_scaler is not None
    ens32 = EnsembleDetector(["efficientnet_b0"], pretrained=False)
    assert TrainStep(ens32).loss_scaler is None
    det16 = PretrainedBackboneDetector("efficientnet_b0", pretrained=False, compute_dtype="fp16")
    assert TrainStep(det16).loss_scaler is not None
