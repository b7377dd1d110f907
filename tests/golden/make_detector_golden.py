"""Golden fixtures for the ``DeepfakeDetector(model_type='rnn')`` seam (``src/detector.py:9-141``), made
by running the REFERENCE ``detector.py`` (build container only; ``cv2`` is an empty stand-in, the
face extractor -- cv2 Haar, out of scope -- is replaced by a stub returning the case's crops).

The seam as SURVEY §3.4 / §8(b) define it: a frame feature extractor ``(N, 3, 224, 224) -> (N, 1280)``
(here the oracle's B0 trunk, ``oracle/b0_cpu.py``, eval mode, portable weights) feeding the
reference ``LogicRNNLSTM(input_size=1280)`` (``src/RNNModel.py``, portable weights).  Recorded:

* ``as_is``   -- ``detect()`` exactly as shipped: ``preprocess_faces`` hands ``torch.from_numpy`` a
  negative-stride view (``[..., ::-1]``, ``detector.py:62-64``) and always fails;
* ``patched`` -- ``preprocess_faces`` with ``.copy()`` added, so the rnn branch runs: features,
  pad/truncate to 10, ``lengths = [num_faces]``, the already-sigmoided output sigmoided again
  (F8b), threshold 0.5, result dict with the explanation text;
* ``no_faces`` -- the extractor finds nothing.

usage: python tests/golden/make_detector_golden.py
"""
from __future__ import annotations

import json
import os
import sys
import types

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import deepfake_amd  # noqa: E402,F401
from deepfake_amd.weights import deterministic_init_  # noqa: E402
from detector_cases import DET_CASES, RNN_CFG, RNN_SEED, TRUNK_SEED, det_faces  # noqa: E402
from oracle import b0_cpu  # noqa: E402


def main():
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    sys.path.insert(0, "/root/reference/src")
    sys.path.insert(0, "/root/reference")
    import detector as D  # noqa: E402
    import RNNModel as R  # noqa: E402

    torch.set_num_threads(8)
    torch.manual_seed(0)
    rnn = R.create_model(dict(RNN_CFG))
    deterministic_init_(rnn, seed=RNN_SEED)
    trunk = b0_cpu.trunk(b0_cpu.EfficientNetB0())
    deterministic_init_(trunk, seed=TRUNK_SEED, prefix="backbone.")
    out = []
    for case in DET_CASES:
        faces = det_faces(case)
        rec = {"name": case["name"], "n": case["n"]}
        for mode in ("as_is", "patched"):
            det = D.DeepfakeDetector(rnn, feature_extractor=trunk, device="cpu", model_type="rnn")
            det.extract_faces = lambda path, max_frames=10, _f=faces: list(_f)
            if mode == "patched":
                orig = D.DeepfakeDetector.preprocess_faces

                def pre(self, fs, _o=orig):
                    if len(fs) == 0:
                        return _o(self, fs)
                    x = np.array(fs, dtype=np.float32) / 255.0
                    return torch.from_numpy(x[..., ::-1].copy()).permute(0, 3, 1, 2)

                det.preprocess_faces = types.MethodType(pre, det)
            rec[mode] = det.detect("clip.mp4")
        out.append(rec)
    json.dump(out, open(os.path.join(HERE, "detector_rnn.json"), "w"), indent=1, sort_keys=True)
    print("detector goldens written to", HERE)


if __name__ == "__main__":
    main()
