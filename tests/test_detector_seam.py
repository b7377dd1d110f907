"""The ``DeepfakeDetector(model_type='rnn')`` seam (``src/detector.py:9-141``): the HIP B0
frame extractor feeding the HIP ``LogicRNNLSTM(1280)``, against tests/golden/detector_rnn.json (the
reference ``detector.py`` run with the oracle trunk and the reference ``LogicRNNLSTM``,
tests/golden/make_detector_golden.py).

* as shipped, ``detect()`` fails on the negative-stride view: same error dict (CPU);
* with the ``.copy()`` fix the rnn branch runs: probability (double sigmoid, F8b) within 2e-6,
  decision, confidence and explanation text equal (GPU, fp32);
* the uint8 handover (BGR gather + strided view, /255 in the stem) gives bit-identical features to
  the reference's float ``preprocess_faces`` tensor (GPU).
"""
import json
import os
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

from detector_cases import DET_CASES, RNN_CFG, RNN_SEED, TRUNK_SEED, det_faces  # noqa: E402

from deepfake_amd.backbone import B0FrameExtractor  # noqa: E402
from deepfake_amd.detector import DeepfakeDetector  # noqa: E402
from deepfake_amd.weights import deterministic_init_  # noqa: E402

GOLD = {r["name"]: r for r in json.load(open(os.path.join(HERE, "golden", "detector_rnn.json")))}


def _modules(device):
    from deepfake_amd.rnn import create_model

    torch.manual_seed(0)
    rnn = create_model(dict(RNN_CFG))
    deterministic_init_(rnn, seed=RNN_SEED)
    fe = B0FrameExtractor()
    deterministic_init_(fe, seed=TRUNK_SEED, prefix="backbone.")
    return rnn.to(device), fe.to(device)


@pytest.mark.parametrize("case", DET_CASES, ids=[c["name"] for c in DET_CASES])
def test_detect_as_shipped(case):
    rnn, fe = _modules("cpu")
    det = DeepfakeDetector(rnn, feature_extractor=fe, device="cpu", model_type="rnn",
                           extract_faces=lambda path, max_frames=10: det_faces(case))
    assert det.detect("clip.mp4") == GOLD[case["name"]]["as_is"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", DET_CASES, ids=[c["name"] for c in DET_CASES])
def test_detect_rnn_branch(cuda, case):
    rnn, fe = _modules(cuda)
    det = DeepfakeDetector(rnn, feature_extractor=fe, device=cuda, model_type="rnn", fix_negative_stride=True,
                           extract_faces=lambda path, max_frames=10: det_faces(case))
    got = det.detect("clip.mp4")
    exp = GOLD[case["name"]]["patched"]
    assert set(got) == set(exp)
    for k, v in exp.items():
        if isinstance(v, float):
            assert abs(got[k] - v) <= 2e-6, (k, got[k], v)
        else:
            assert got[k] == v, k


@pytest.mark.gpu
def test_uint8_handover_bit_identical(cuda):
    rnn, fe = _modules(cuda)
    det = DeepfakeDetector(rnn, feature_extractor=fe, device=cuda, model_type="rnn", fix_negative_stride=True)
    faces = det_faces({"name": "three_faces", "n": 3})
    with torch.no_grad():
        a = fe(det._frames(faces))
        b = fe(det.preprocess_faces(faces).to(cuda))
    assert det._frames(faces).dtype == torch.uint8
    assert torch.equal(a, b)
