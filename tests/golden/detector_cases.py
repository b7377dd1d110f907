"""Case definitions shared by tests/golden/make_detector_golden.py and tests/test_detector_seam.py
(data only: face-crop counts and the portable weight seeds)."""
from __future__ import annotations

import numpy as np

from deepfake_amd.weights import hash_uniform

RNN_CFG = {"input_size": 1280, "hidden_size": 64, "num_layers": 2, "dropout": 0.5}
RNN_SEED = 17
TRUNK_SEED = 19
DET_CASES = [{"name": "three_faces", "n": 3}, {"name": "ten_faces", "n": 10}, {"name": "twelve_faces", "n": 12},
             {"name": "no_faces", "n": 0}]


def det_faces(case, size=224):
    """BGR uint8 face crops (what cv2 hands detector.extract_faces)."""
    n = int(case["n"])
    out = []
    for i in range(n):
        u = hash_uniform(23 + i, "det_faces/" + case["name"], size * size * 3)
        out.append(((u + 1.0) * 127.5).astype(np.uint8).reshape(size, size, 3))
    return out
