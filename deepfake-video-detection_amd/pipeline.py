"""Input pipeline in front of the hot path: the ``.npz`` face-crop feed, the
collate sampling rules, and the uint8 -> device handover.

Reference chain: ``data_prepare.py`` writes one ``.npz`` per video ``{faces: uint8 (N,224,224,3),
label}`` (``:278-281``); ``VideoFacesDataset.__getitem__`` loads it and infers the label from the
file name when absent (``dataset.py:43-81``); ``collate_batch_cnn_lstm`` / ``collate_batch``
(``train.py:38-61, 62-100``) sample ``linspace(0, M-1, T).astype(int)`` frames or pad with the last
frame (zeros if M == 0), stack, permute and divide by 255 ON THE HOST, then ``.to(device)``.

Here the index rule stays on the host (a few integers per clip), the crops cross PCIe as uint8
(4x fewer bytes than the fp32 batch) and the gather + ``/255`` run on the device
(``torch.ops.dfd.collate_frames`` -> ``dfd_collate_frames``, ``csrc/k_input.hip``), bit-identical to the reference's float batch.  For
the B0 detector the uint8 batch itself can be handed to the model (normalised in the stem).
"""
from __future__ import annotations

from pathlib import Path

import numpy as np
import torch

from . import _lib, ops  # noqa: F401  (registers torch.ops.dfd.*)
from .detector import normalize_adjacency


def infer_label(fname: str) -> int:
    """``VideoFacesDataset.infer_label`` (dataset.py:43-49)."""
    s = fname.lower()
    if "fake" in s or "deepfake" in s:
        return 1
    if "real" in s or "original" in s:
        return 0
    return -1


class NpzFaces:
    """``VideoFacesDataset`` without the (torchvision) augmentation: one ``.npz`` per video; samples are
    ``{'faces': uint8 (N,H,W,3), 'label': int, 'file': name}`` (dataset.py:51-81).  Loaded with
    ``allow_pickle=False``.  The reference's eval transform (``T.Resize(image_size)``) is the identity
    on the 224x224 crops data_prepare.py writes; other sizes are refused instead of resized."""

    def __init__(self, data_dir, image_size=(224, 224), recursive=False):
        d = Path(data_dir)
        self.files = sorted(d.rglob("*.npz") if recursive else d.glob("*.npz"))
        self.image_size = tuple(image_size)

    def __len__(self):
        return len(self.files)

    def __getitem__(self, idx):
        p = self.files[idx]
        with np.load(p, allow_pickle=False) as data:
            faces = data["faces"]
            label = int(np.array(data["label"]).item()) if "label" in data else infer_label(p.name)
        if label == -1:
            raise ValueError(f"Could not infer label from filename: {p.name}. "
                             "Expected 'fake'/'real' (or 'deepfake'/'original') in the filename.")
        if faces.ndim != 4 or faces.dtype != np.uint8:
            raise ValueError(f"{p.name}: expected uint8 faces (N, H, W, C), got {faces.dtype} {faces.shape}")
        if faces.shape[0] and tuple(faces.shape[1:3]) != self.image_size:
            raise ValueError(f"{p.name}: faces are {faces.shape[1:3]}, expected {self.image_size} (resize is not "
                             "part of the device pipeline)")
        return {"faces": faces, "label": label, "file": str(p.name)}


def select_frames(m: int, max_frames: int = 16) -> np.ndarray:
    """Frame indices of one clip (train.py:38-61): ``linspace`` when M >= T, else 0..M-1 then the last
    frame repeated; -1 = an all-zero frame (M == 0)."""
    if m >= max_frames:
        return np.linspace(0, m - 1, max_frames).astype(int)
    if m == 0:
        return np.full(max_frames, -1, dtype=np.int64)
    return np.concatenate([np.arange(m), np.full(max_frames - m, m - 1)]).astype(np.int64)


def collate_clips(batch, max_frames=16, image_size=(224, 224), device="cuda", out="float"):
    """Device collate of ``[{'faces': uint8 (M,H,W,3), 'label': ...}]`` -> ``(x (B,T,3,H,W), labels)``.

    ``out="float"``: fp32 ``v / 255`` (exactly ``collate_batch_cnn_lstm``'s tensor, channels-last
    strides); ``out="uint8"``: the raw crops, for a B0 detector that normalises them in its stem.
    Which normalisation the stem applies is the DETECTOR's ``input_normalization``: the reference
    TRAINING feed is ``/255`` only (src/train.py:59), so a training model fed these uint8 batches must
    be built with ``input_normalization="unit"`` to see the reference trainer's tensor; the default
    ``"imagenet"`` is the serving feed (app.py:2084-2085)."""
    dev = torch.device(device)
    if dev.type != "cuda":
        raise _lib.DFDError("collate_clips runs on a HIP device; the MI355X path has no CPU fallback")
    h, w = image_size
    frame_bytes = h * w * 3
    srcs, sel, labels, base = [], [], [], 0
    for item in batch:
        faces = np.asarray(item["faces"])
        m = int(faces.shape[0])
        if m and (faces.dtype != np.uint8 or tuple(faces.shape[1:]) != (h, w, 3)):
            raise ValueError(f"expected uint8 faces (M, {h}, {w}, 3), got {faces.dtype} {faces.shape}")
        idx = select_frames(m, max_frames)
        sel.append(np.where(idx >= 0, idx + base, -1))
        if m:
            srcs.append(faces.reshape(m, frame_bytes))
        base += m
        labels.append(item["label"] if item["label"] is not None else -1)
    b = len(batch)
    sel = torch.from_numpy(np.concatenate(sel).astype(np.int64)) if b else torch.zeros(0, dtype=torch.int64)
    host = np.ascontiguousarray(np.concatenate(srcs)) if srcs else np.zeros((1, frame_bytes), np.uint8)
    src = torch.from_numpy(host).pin_memory().to(dev, non_blocking=True)
    sel_d = sel.pin_memory().to(dev, non_blocking=True)
    o = torch.ops.dfd.collate_frames(src, sel_d, [h, w, 3], out == "float").view(b, max_frames, h, w, 3)
    # (the pinned staging and the device source are stream-ordered: torch's allocators keep them
    # until the copy and the gather have run)
    return o.permute(0, 1, 4, 2, 3), torch.tensor(labels, dtype=torch.long)


def collate_graph_clips(batch, max_nodes=16, image_size=(224, 224), device="cuda"):
    """``collate_batch`` (train.py:62-100): the same frames plus a chain graph over the nodes,
    ``normalize_adjacency`` per clip."""
    x, labels = collate_clips(batch, max_frames=max_nodes, image_size=image_size, device=device)
    n = max_nodes
    a = np.zeros((n, n), dtype=np.float32)
    for i in range(n - 1):
        a[i, i + 1] = a[i + 1, i] = 1.0
    a_norm = torch.from_numpy(np.stack([normalize_adjacency(a) for _ in range(len(batch))])).float().to(device)
    return x, a_norm, labels
