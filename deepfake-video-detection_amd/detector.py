"""``DeepfakeDetector`` (``src/detector.py:9-167``) on the HIP modules -- the third drop-in seam
(SURVEY F2, §3.4): a frame feature extractor (``backbone.B0FrameExtractor``: crops -> pooled B0
features) feeding ``rnn.LogicRNNLSTM(input_size=1280)``.

The reference class is usable unchanged with these modules (``feature_extractor(Tensor(N,3,224,224))
-> (N,1280)``, ``model(Tensor(1,10,F), Tensor([n])) -> (1,1)``).  This restatement exists so the
seam can be exercised without the reference tree (tests on the GPU box) and so the crops can stay
uint8 up to the stem kernel: the reference's ``/255``, BGR->RGB flip and HWC->CHW
(``preprocess_faces``, ``:54-66``) become a channel gather + a strided uint8 view, normalised
inside the stem (``input_normalization="unit"``), bit-identical to the float path.

Reference behaviour kept, quirks included:

* ``detect()`` -- the shipped ``preprocess_faces`` hands ``torch.from_numpy`` a negative-stride
  view and always raises, so ``detect()`` returns ``{'success': False, 'error': <torch message>,
  ...}``.  ``DeepfakeDetector(..., fix_negative_stride=True)`` runs the intended path
  (the reference with ``.copy()`` added).
* the rnn branch pads/truncates the features to 10, passes ``lengths=[num_faces]`` (un-clamped),
  and applies ``sigmoid`` to ``LogicRNNLSTM``'s already-sigmoided output (F8b);
* face extraction (cv2 Haar, ``:21-52``) is out of scope: inject ``extract_faces`` (a callable
  ``(video_path, max_frames) -> list of BGR uint8 crops``) or call ``detect_faces``.
The gcn branch (``:101-118``) belongs to the ViT+GCN model (``vit_gcn.DeepfakeModel``) and follows
the same structure.
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np
import torch


def normalize_adjacency(a: np.ndarray) -> np.ndarray:
    """``normalize_adjacency`` (src/utils.py:95-104): D^-1/2 (A + I) D^-1/2 in float32."""
    a = a.copy().astype(np.float32)
    a = a + np.eye(a.shape[0], dtype=a.dtype)
    with np.errstate(divide="ignore"):
        d = np.power(np.sum(a, axis=1), -0.5)
    d[np.isinf(d)] = 0.0
    dm = np.diag(d)
    return dm @ a @ dm


def chain_adjacency(n: int) -> np.ndarray:
    """The detector's chain graph over the faces (``detector.py:104-111``), normalised."""
    a = np.zeros((n, n), dtype=np.float32)
    for i in range(n - 1):
        a[i, i + 1] = a[i + 1, i] = 1.0
    return normalize_adjacency(a)


def generate_explanation(is_fake: int, confidence: float, num_faces: int) -> str:
    """``generate_explanation`` (src/detector.py:143-167), verbatim output text."""
    if is_fake == 1:
        return (
            f"🚨 **LIKELY DEEPFAKE DETECTED** (confidence: {confidence*100:.1f}%)\n\n"
            f"The model detected {num_faces} face(s) in the video with synthetic manipulation patterns. "
            f"Key indicators:\n"
            f"- Facial feature artifacts and inconsistencies\n"
            f"- Unnatural eye movement or blinking patterns\n"
            f"- Audio-visual misalignment\n"
            f"- Lighting and shadow inconsistencies\n\n"
            f"⚠️ This is a probabilistic assessment. Manual review recommended for critical decisions."
        )
    confidence_real = 1.0 - confidence
    return (
        f"✅ **LIKELY AUTHENTIC** (confidence: {confidence_real*100:.1f}%)\n\n"
        f"The model detected {num_faces} face(s) in the video with natural characteristics. "
        f"Key indicators:\n"
        f"- Natural facial features and expressions\n"
        f"- Consistent eye movement and blinking\n"
        f"- Proper audio-visual synchronization\n"
        f"- Realistic lighting and shadows\n\n"
        f"✓ Video appears authentic based on analyzed characteristics."
    )


class DeepfakeDetector:
    SEQ_LEN = 10  # detector.py:92-96

    def __init__(self, model, feature_extractor=None, device="cpu", model_type="gcn", extract_faces=None,
                 fix_negative_stride=False):
        self.model = model
        self.feature_extractor = feature_extractor
        self.device = device
        self.model_type = model_type
        self._extract = extract_faces
        self.fix_negative_stride = fix_negative_stride
        self.model.eval()
        if feature_extractor:
            self.feature_extractor.eval()

    def extract_faces(self, video_path: str, max_frames=10):
        if self._extract is None:
            print("Error extracting faces: no face extractor configured (cv2 Haar detection is out of scope)")
            return []
        try:
            return list(self._extract(video_path, max_frames=max_frames))
        except Exception as e:
            print(f"Error extracting faces: {e}")
            return []

    def preprocess_faces(self, faces: List[np.ndarray]) -> torch.Tensor:
        """Float path of the reference (``:54-66``), quirk included unless fix_negative_stride."""
        if len(faces) == 0:
            return torch.zeros(1, 3, 224, 224)
        faces_np = np.array(faces, dtype=np.float32) / 255.0
        faces_np = faces_np[..., ::-1]
        if self.fix_negative_stride:
            faces_np = faces_np.copy()
        return torch.from_numpy(faces_np).permute(0, 3, 1, 2)

    def _frames(self, faces):
        """Crops -> the feature extractor's input on the device.  The HIP trunk takes the uint8 crops:
        BGR -> RGB is a channel gather, HWC -> CHW a strided view, /255 runs in the stem."""
        fe = self.feature_extractor
        if getattr(fe, "accepts_uint8_frames", False) and getattr(fe, "input_normalization", None) == "unit":
            if not self.fix_negative_stride:  # reproduce the reference's failure (F8a) exactly
                torch.from_numpy(np.zeros((1, 1, 2), dtype=np.float32)[..., ::-1])
            u8 = torch.from_numpy(np.ascontiguousarray(np.stack(faces))).to(self.device)
            rgb = u8.index_select(3, torch.tensor([2, 1, 0], device=u8.device))
            return rgb.permute(0, 3, 1, 2)
        return self.preprocess_faces(faces).to(self.device)

    def detect(self, video_path: str) -> Dict:
        return self._detect(lambda: self.extract_faces(video_path, max_frames=10))

    def detect_faces(self, faces: List[np.ndarray]) -> Dict:
        """``detect`` on already-extracted BGR crops."""
        return self._detect(lambda: list(faces))

    def _detect(self, get_faces) -> Dict:
        try:
            faces = get_faces()
            num_faces = len(faces)
            if num_faces == 0:
                return {"success": False, "error": "No faces detected in video", "num_faces": 0, "is_fake": None,
                        "confidence": 0.0}
            faces_tensor = self._frames(faces)
            with torch.no_grad():
                if self.model_type == "rnn":
                    feats = self.feature_extractor(faces_tensor)  # (N, F)
                    if feats.shape[0] < self.SEQ_LEN:
                        pad = self.SEQ_LEN - feats.shape[0]
                        feats = torch.cat([feats, torch.zeros(pad, feats.shape[1], device=feats.device)])
                    else:
                        feats = feats[: self.SEQ_LEN]
                    feats = feats.unsqueeze(0)
                    output = self.model(feats, torch.tensor([num_faces], device=feats.device))
                    probs = torch.sigmoid(output).squeeze().cpu().numpy()  # F8b: a second sigmoid
                else:
                    n = faces_tensor.shape[0]
                    a = torch.from_numpy(chain_adjacency(n)).float().unsqueeze(0).to(faces_tensor.device)
                    output = self.model(faces_tensor.float().unsqueeze(0), a)
                    if output.dim() == 1:
                        probs = torch.sigmoid(output).squeeze().cpu().numpy()
                    else:
                        probs = torch.softmax(output, dim=1)[0, 1].cpu().numpy()
            is_fake_prob = (float(probs) if isinstance(probs, np.ndarray) and probs.ndim == 0
                            else float(probs.mean()) if isinstance(probs, np.ndarray) else float(probs))
            is_fake_pred = 1 if is_fake_prob >= 0.5 else 0
            confidence = is_fake_prob if is_fake_pred == 1 else (1.0 - is_fake_prob)
            return {"success": True, "error": None, "is_fake": is_fake_pred, "is_fake_prob": is_fake_prob,
                    "confidence": confidence, "num_faces": num_faces,
                    "explanation": generate_explanation(is_fake_pred, is_fake_prob, num_faces)}
        except Exception as e:
            return {"success": False, "error": str(e), "num_faces": 0, "is_fake": None, "confidence": 0.0}
