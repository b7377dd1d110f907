"""Serving on the HIP detector: the pretrained branch of ``app.predict_video`` (``app.py:2027-2223``).

``FrameClassifierService`` is what ``app.load_model(path, 'pretrained')`` + ``predict_video`` do
around the model -- minus face extraction (MTCNN/Haar + video decode are out of scope; the caller
passes the uint8 face crops ``extract_faces_from_video`` returns, or injects that function):

* ``MAX_FRAMES`` (default 8, clamped 1..64) and ``MIN_FACES`` (default 2) gates;
* the crops go to the device as uint8 (1 B/px over PCIe instead of 4) and the app's
  ``/255`` + ImageNet normalisation (``:2084-2085``, ``imagenet_normalize`` ``:1772-1780``) runs
  inside the stem kernel, bit-identical to normalising first (``tests/test_serving.py``);
* ``softmax`` over the 2 logits, fake-class index (``FAKE_CLASS_INDEX`` env > checkpoint
  metadata > 1, ``:1833-1869``), threshold (``calibration_best.json`` next to the checkpoint >
  ``DETECT_FAKE_THRESHOLD`` > 0.5, extreme values ignored unless
  ``ALLOW_EXTREME_CALIBRATION_THRESHOLD``, ``:2096-2109``), borderline / low-confidence abstain
  (``DETECT_ABSTAIN_MARGIN``, ``DETECT_ABSTAIN_CONF``, ``:2173-2210``) and the result dict with
  the same keys, values and descriptions; any exception becomes ``{'error': str(e)}`` (``:2320``).

The enhanced decision agent (``:2118-2171``) is ensemble-only and out of scope: ``enhanced_agent``
is always None, as in the app when it is disabled.

``predict_batch`` is the batched multi-video variant: videos with the same face
count go through ONE forward of shape (videos, T, 3, H, W); in eval mode the clips do not
interact, so each result equals the single-video one.
"""
from __future__ import annotations

import json
import os
from pathlib import Path

import numpy as np
import torch

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


# ------------------------------------------------------------------ env helpers (app.py:352, 1802-1906)
def _safe_int(x):
    try:
        return int(x)
    except Exception:
        return None


def _env_float(name):
    v = os.environ.get(name)
    if v is None:
        return None
    v = str(v).strip()
    if not v:
        return None
    try:
        return float(v)
    except Exception:
        return None


def _env_int(name):
    v = os.environ.get(name)
    if v is None:
        return None
    v = str(v).strip()
    if not v:
        return None
    return _safe_int(v)


def _env_flag(name):
    return str(os.environ.get(name, "")).strip().lower() in ("1", "true", "yes", "y")


def fake_class_index(num_classes=2, load_stats=None):
    nc = max(1, int(num_classes))
    idx = _env_int("FAKE_CLASS_INDEX")
    if idx is not None and 0 <= idx < nc:
        return int(idx)
    det = (load_stats or {}).get("fake_class_index_detected")
    if det is not None:
        d = _safe_int(det)
        if d is not None and 0 <= d < nc:
            return d
    return 1 if nc > 1 else 0


def threshold_fallback(default=0.5):
    t = _env_float("DETECT_FAKE_THRESHOLD")
    if t is not None and 0.0 <= float(t) <= 1.0:
        return float(t)
    return float(default)


def calibration_threshold(checkpoint_path):
    """``best_thr_accuracy`` of calibration_best.json next to the checkpoint (app.py:1783-1799)."""
    if not checkpoint_path:
        return None
    try:
        cand = Path(checkpoint_path).parent / "calibration_best.json"
        if cand.exists():
            thr = json.loads(cand.read_text(encoding="utf-8")).get("best_thr_accuracy")
            if thr is not None:
                t = float(thr)
                return t if 0.0 <= t <= 1.0 else None
    except Exception:
        return None
    return None


def max_frames_setting():
    try:
        m = int(os.environ.get("MAX_FRAMES", "8"))
    except Exception:
        m = 8
    return max(1, min(64, int(m)))


def imagenet_normalize(frames: torch.Tensor) -> torch.Tensor:
    """``app.imagenet_normalize`` (float frames in [0,1], (T,C,H,W) or (B,T,C,H,W))."""
    mean = torch.tensor(IMAGENET_MEAN, device=frames.device, dtype=frames.dtype)
    std = torch.tensor(IMAGENET_STD, device=frames.device, dtype=frames.dtype)
    if frames.dim() == 4:
        return (frames - mean.view(1, 3, 1, 1)) / std.view(1, 3, 1, 1)
    if frames.dim() == 5:
        return (frames - mean.view(1, 1, 3, 1, 1)) / std.view(1, 1, 3, 1, 1)
    raise ValueError(f"Unsupported frames shape for normalization: {tuple(frames.shape)}")


def decide(logits_row: torch.Tensor, num_faces: int, checkpoint_path=None, load_stats=None, ensemble=False):
    """Post-processing of ONE video's logits (app.py:2090-2223): probabilities, threshold, abstain
    rules, result dict."""
    try:
        abstain_conf = float(os.environ.get("DETECT_ABSTAIN_CONF", "0.60"))
    except Exception:
        abstain_conf = 0.60
    try:
        abstain_margin = float(os.environ.get("DETECT_ABSTAIN_MARGIN", "0.0"))
    except Exception:
        abstain_margin = 0.0
    abstain_margin = max(0.0, min(0.5, float(abstain_margin)))

    probs = torch.softmax(logits_row.detach().float().cpu().reshape(1, -1), dim=1)
    nc = int(probs.shape[1])
    fake_idx = fake_class_index(nc, load_stats)
    real_idx = (1 - int(fake_idx)) if nc == 2 else 0
    prob_fake = float(probs[0, int(fake_idx)].item())
    prob_real = float(probs[0, int(real_idx)].item())
    thr = calibration_threshold(checkpoint_path)
    thr = threshold_fallback(0.5) if thr is None else float(thr)
    thr = float(threshold_fallback(thr))
    if not _env_flag("ALLOW_EXTREME_CALIBRATION_THRESHOLD") and (float(thr) < 0.05 or float(thr) > 0.95):
        thr = 0.5
    is_fake = bool(prob_fake >= float(thr))
    pred_class = 1 if is_fake else 0
    confidence = float(prob_fake if is_fake else prob_real)
    description = (f"Pretrained detector (thr={thr:.2f})" if not ensemble
                   else f"Ensemble pretrained detector (thr={thr:.2f})")
    agent_payload = None
    if abstain_margin > 0.0 and abs(float(prob_fake) - float(thr)) <= float(abstain_margin):
        return {"prediction": "Uncertain", "verdict_yes_no": "Unsure",
                "description": (f"Borderline score (prob_fake={prob_fake * 100:.1f}%, thr={thr:.2f} ± "
                                f"{abstain_margin:.2f}). Manual review recommended.\n\n" + (description or "")),
                "pred_class": None, "confidence": float(confidence), "prob_real": float(prob_real),
                "prob_fake": float(prob_fake), "num_faces": int(num_faces), "threshold": float(thr),
                "enhanced_agent": agent_payload, "abstained": True}
    if confidence < float(abstain_conf):
        return {"prediction": "Uncertain", "verdict_yes_no": "Unsure",
                "description": (f"Low confidence ({confidence * 100:.1f}%). This video may be out-of-domain "
                                "(different compression, face quality, lighting, or manipulation type). Manual "
                                "review recommended.\n\n" + (description or "")),
                "pred_class": None, "confidence": float(confidence), "prob_real": float(prob_real),
                "prob_fake": float(prob_fake), "num_faces": int(num_faces), "threshold": float(thr),
                "enhanced_agent": agent_payload, "abstained": True}
    return {"prediction": "Deepfake" if pred_class == 1 else "Real",
            "verdict_yes_no": "Yes" if pred_class == 1 else "No", "description": description,
            "pred_class": int(pred_class), "confidence": float(confidence), "prob_real": float(prob_real),
            "prob_fake": float(prob_fake), "num_faces": int(num_faces), "threshold": float(thr),
            "enhanced_agent": agent_payload}


def _too_few(num_faces):
    try:
        min_faces = int(os.environ.get("MIN_FACES", "2"))
    except Exception:
        min_faces = 2
    min_faces = max(1, int(min_faces))
    if num_faces < min_faces:
        return {"prediction": "Uncertain", "verdict_yes_no": "Unsure",
                "description": (f"Not enough faces/frames detected for a stable decision (num_faces={num_faces}, "
                                f"min_faces={min_faces}). Try a clearer face shot, better lighting, or a longer clip."),
                "pred_class": None, "confidence": None, "prob_real": None, "prob_fake": None,
                "num_faces": int(num_faces), "abstained": True}
    return None


class FrameClassifierService:
    """Model + checkpoint context of the app's pretrained serving path on one device."""

    def __init__(self, model, checkpoint_path=None, load_stats=None, device=None):
        self.model = model.eval()
        self.checkpoint_path = checkpoint_path
        self.load_stats = load_stats or {}
        self.device = torch.device(device) if device is not None else next(model.parameters()).device

    @classmethod
    def from_checkpoint(cls, path, device="cuda", compute_dtype="fp32"):
        from .checkpoint import load_pretrained

        model, stats = load_pretrained(path, device=device, compute_dtype=compute_dtype)
        return cls(model, checkpoint_path=str(path), load_stats={**stats, "checkpoint": str(path)}, device=device)

    # -- tensor handover (app.py:2084-2086)
    def _frames(self, faces_list):
        """(V, T, H, W, 3) uint8 crops -> the model's input (V, T, 3, H, W) on the device."""
        u8 = torch.from_numpy(np.ascontiguousarray(np.stack(faces_list))).to(self.device, non_blocking=True)
        x = u8.permute(0, 1, 4, 2, 3)  # channels-last strides, as the app's permute
        if getattr(self.model, "accepts_uint8_frames", False):
            return x  # normalised inside the stem kernel
        return imagenet_normalize(x.float() / 255.0)  # a model without the fused input path

    @torch.no_grad()
    def _logits(self, faces_list):
        out = self.model(self._frames(faces_list))
        logits = out[0] if isinstance(out, tuple) else out
        return logits.float().cpu()

    def predict_faces(self, faces: np.ndarray) -> dict:
        try:
            num_faces = int(len(faces))
            if num_faces == 0:
                return {"error": "No faces detected in video"}
            few = _too_few(num_faces)
            if few is not None:
                return few
            logits = self._logits([faces])
            return decide(logits[0], num_faces, self.checkpoint_path, self.load_stats,
                          ensemble=hasattr(self.model, "models"))
        except Exception as e:
            return {"error": str(e)}

    def predict_video(self, video_path, extract_faces) -> dict:
        """``predict_video`` with the face extractor injected (``extract_faces(path, max_frames=)``)."""
        try:
            faces = extract_faces(video_path, max_frames=max_frames_setting())
        except Exception as e:
            return {"error": str(e)}
        return self.predict_faces(faces)

    def predict_batch(self, faces_per_video) -> list:
        """Batched multi-video serving: one forward per group of videos with equal face count."""
        results = [None] * len(faces_per_video)
        groups = {}
        for i, faces in enumerate(faces_per_video):
            n = int(len(faces))
            if n == 0:
                results[i] = {"error": "No faces detected in video"}
                continue
            few = _too_few(n)
            if few is not None:
                results[i] = few
                continue
            groups.setdefault((n,) + tuple(np.shape(faces)[1:]), []).append(i)
        for _, idxs in groups.items():
            try:
                logits = self._logits([faces_per_video[i] for i in idxs])
                for j, i in enumerate(idxs):
                    results[i] = decide(logits[j], int(len(faces_per_video[i])), self.checkpoint_path,
                                        self.load_stats, ensemble=hasattr(self.model, "models"))
            except Exception as e:
                for i in idxs:
                    results[i] = {"error": str(e)}
        return results
