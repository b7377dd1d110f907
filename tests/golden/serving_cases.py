"""Case definitions shared by tests/golden/make_serving_golden.py (which runs the reference app on
them) and tests/test_serving.py (which runs this package on them).  Data only: face-crop shapes,
stub logits, environment settings, calibration files and checkpoint layouts."""
from __future__ import annotations

import numpy as np
import torch

from deepfake_amd.weights import deterministic_init_, hash_uniform

SERVE_CASES = [
    {"name": "no_faces", "n": 0, "logits": [0.0, 1.0]},
    {"name": "one_face", "n": 1, "logits": [0.0, 1.0]},
    {"name": "one_face_min1", "n": 1, "logits": [0.0, 2.0], "env": {"MIN_FACES": "1"}},
    {"name": "fake_high", "n": 8, "logits": [-1.0, 1.5]},
    {"name": "real_high", "n": 8, "logits": [2.0, -0.5]},
    {"name": "low_conf", "n": 5, "logits": [0.0, 0.2]},
    {"name": "margin", "n": 6, "logits": [0.0, 0.3], "env": {"DETECT_ABSTAIN_MARGIN": "0.1"}},
    {"name": "margin_clamped", "n": 6, "logits": [0.0, 0.3], "env": {"DETECT_ABSTAIN_MARGIN": "0.9"}},
    {"name": "thr_env", "n": 4, "logits": [0.0, 1.0], "env": {"DETECT_FAKE_THRESHOLD": "0.7"}},
    {"name": "thr_env_real", "n": 4, "logits": [0.0, 1.0], "env": {"DETECT_FAKE_THRESHOLD": "0.8"}},
    {"name": "thr_env_bad", "n": 4, "logits": [0.0, 1.0], "env": {"DETECT_FAKE_THRESHOLD": "1.7"}},
    {"name": "calib", "n": 4, "logits": [0.5, 0.0], "calibration": {"best_thr_accuracy": 0.3},
     "env": {"DETECT_ABSTAIN_CONF": "0.3"}},
    {"name": "calib_extreme", "n": 4, "logits": [0.5, 0.0], "calibration": {"best_thr_accuracy": 0.99}},
    {"name": "calib_extreme_allowed", "n": 4, "logits": [-3.0, 3.0], "calibration": {"best_thr_accuracy": 0.99},
     "env": {"ALLOW_EXTREME_CALIBRATION_THRESHOLD": "yes"}},
    {"name": "calib_out_of_range", "n": 4, "logits": [-1.0, 1.0], "calibration": {"best_thr_accuracy": 1.5}},
    {"name": "fake_idx0", "n": 3, "logits": [2.0, -1.0], "env": {"FAKE_CLASS_INDEX": "0"}},
    {"name": "fake_idx_bad", "n": 3, "logits": [2.0, -1.0], "env": {"FAKE_CLASS_INDEX": "7"}},
    {"name": "max_frames_big", "n": 3, "logits": [0.0, 1.0], "env": {"MAX_FRAMES": "100"}},
    {"name": "max_frames_bad", "n": 3, "logits": [0.0, 1.0], "env": {"MAX_FRAMES": "abc"}},
    {"name": "max_frames_zero", "n": 3, "logits": [0.0, 1.0], "env": {"MAX_FRAMES": "0"}},
    {"name": "abstain_conf_bad", "n": 3, "logits": [0.0, 0.9], "env": {"DETECT_ABSTAIN_CONF": "x"}},
    {"name": "model_raises", "n": 3, "logits": [0.0, 1.0], "model_raises": True},
]


def faces_for(case, size=16):
    n = int(case["n"])
    u = hash_uniform(11, "faces/" + case["name"], max(1, n * size * size * 3))
    return ((u[: n * size * size * 3] + 1.0) * 127.5).astype(np.uint8).reshape(n, size, size, 3)


# ------------------------------------------------------------------------------ checkpoints
CKPT_SEED = 41
CKPT_VARIANTS = ["raw", "model_state", "state_dict_module", "model_prefix_meta", "partial", "shape_mismatch",
                 "ensemble_prefix"]


def reference_state_dict():
    """state_dict of the oracle detector (the reference's keys) with the portable weights."""
    from oracle.detector_cpu import DetectorCPU

    m = DetectorCPU(dropout_rate=0.5)
    deterministic_init_(m, seed=CKPT_SEED)
    return {k: v.clone() for k, v in m.state_dict().items()}


def ckpt_variant(name):
    """The checkpoint object of one layout (what torch.save writes to disk)."""
    sd = reference_state_dict()
    if name == "raw":  # EnsembleTrainer._save_checkpoint: torch.save(model.state_dict()) (ensemble_trainer.py:549-571)
        return sd
    if name == "model_state":  # train.py:398-411 dict format (+ class map metadata)
        return {"epoch": 3, "model_state": sd, "optimizer_state": {}, "best_f1": 0.5,
                "class_to_idx": {"real": 0, "fake": 1}}
    if name == "state_dict_module":  # DataParallel-prefixed keys
        return {"state_dict": {"module." + k: v for k, v in sd.items()}}
    if name == "model_prefix_meta":
        return {"model_state": {"model.module." + k: v for k, v in sd.items()},
                "meta": {"classes": ["fake", "real"]}}
    if name == "partial":  # < 80 % of the model's keys -> refused
        keys = sorted(sd)
        return {k: sd[k] for i, k in enumerate(keys) if i % 3 != 0}
    if name == "shape_mismatch":  # a 3-class head: fc2 skipped by the shape filter
        sd = dict(sd)
        sd["fc2.weight"] = torch.zeros(3, 256)
        sd["fc2.bias"] = torch.zeros(3)
        return sd
    if name == "ensemble_prefix":  # an EnsembleDetector checkpoint given as a single detector
        return {"models.0." + k: v for k, v in sd.items()}
    raise KeyError(name)


def ckpt_frames():
    n = 1 * 3 * 3 * 64 * 64
    u = (hash_uniform(43, "ckpt_frames", n) + 1.0) * 0.5
    x = torch.from_numpy(u.reshape(1, 3, 3, 64, 64))
    mean = torch.tensor([0.485, 0.456, 0.406]).view(1, 1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225]).view(1, 1, 3, 1, 1)
    return ((x - mean) / std).float()
