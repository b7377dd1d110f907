"""Checkpoint I/O with the reference's formats and loader semantics.

The unchanged ``app.load_model`` (``app.py:1327-1769``) constructs ``PretrainedBackboneDetector``
and loads through its own helpers; the build's module has the same ``state_dict`` keys and
shapes, so that works as is.  This module restates those helpers for callers that load without
the app (training resume, the serving service below, tests):

* ``extract_state_dict``       -- ``ckpt.get('model_state') or ckpt.get('state_dict') or ckpt`` (``:1336-1339``)
* ``detect_fake_class_index``  -- class-map metadata scan (``:1342-1405``)
* ``normalize_state_dict_keys`` -- strip ``module.`` / ``model.`` / ``net.`` repeatedly (``:1413-1432``)
* ``load_stats``               -- matched / mismatched / missing / unexpected / match_ratio (``:1490-1528``)
* ``safe_load_state_dict``     -- load only shape-matching keys, ``strict=False`` (``:1476-1488``)
* ``load_pretrained``          -- the ``'pretrained'`` branch of ``load_model``: backbone inference,
  stats, safe load, the ``match_ratio < 0.80`` refusal (``:1681-1749``)

and the trainers' save formats: a raw ``state_dict`` (``EnsembleTrainer._save_checkpoint``,
``src/ensemble_trainer.py:549-571``) and ``{'epoch', 'model_state', 'optimizer_state',
'scheduler_state', 'metrics', 'best_f1'}`` (``src/train.py:398-411``).  Data-parallel training
saves rank 0's module without a ``module.`` prefix (the loader would strip it anyway).
Checkpoints are read with ``torch.load(..., weights_only=True)``: tensors and plain containers only.
"""
from __future__ import annotations

from pathlib import Path

import torch

PREFIXES = ("module.", "model.", "net.")


def extract_state_dict(ckpt):
    if isinstance(ckpt, dict):
        return ckpt.get("model_state") or ckpt.get("state_dict") or ckpt
    return ckpt


def detect_fake_class_index(obj):
    """Index of the 'fake' class from checkpoint metadata, or None (app.py:1342-1405)."""
    try:
        if not isinstance(obj, dict):
            return None

        def norm(s):
            return str(s).strip().lower().replace("-", "_").replace(" ", "_")

        for key in ("class_to_idx", "class2idx", "label_to_idx", "label2idx"):
            m = obj.get(key)
            if isinstance(m, dict):
                for k, v in m.items():
                    kk = norm(k)
                    if "fake" in kk or "deepfake" in kk:
                        try:
                            return int(v)
                        except Exception:
                            continue
        for key in ("idx_to_class", "idx2class", "idx_to_label", "idx2label"):
            m = obj.get(key)
            if isinstance(m, dict):
                for k, v in list(m.items()):
                    try:
                        idx = int(k)
                    except Exception:
                        continue
                    vv = norm(v)
                    if "fake" in vv or "deepfake" in vv:
                        return idx
            elif isinstance(m, (list, tuple)):
                for idx, v in enumerate(list(m)):
                    vv = norm(v)
                    if "fake" in vv or "deepfake" in vv:
                        return idx
        for key in ("classes", "class_names", "labels", "label_names"):
            m = obj.get(key)
            if isinstance(m, (list, tuple)):
                for idx, v in enumerate(list(m)):
                    vv = norm(v)
                    if "fake" in vv or "deepfake" in vv:
                        return idx
        for key in ("meta", "metadata"):
            sub = obj.get(key)
            if isinstance(sub, dict):
                out = detect_fake_class_index(sub)
                if out is not None:
                    return out
    except Exception:
        return None
    return None


def normalize_state_dict_keys(sd):
    if not isinstance(sd, dict) or not sd:
        return sd
    out = {}
    for k, v in sd.items():
        if not isinstance(k, str):
            out[k] = v
            continue
        nk, changed = k, True
        while changed:
            changed = False
            for pfx in PREFIXES:
                if nk.startswith(pfx):
                    nk = nk[len(pfx):]
                    changed = True
        out[nk] = v
    return out


def _shape_ok(msd, k, v):
    try:
        return tuple(msd[k].shape) == tuple(v.shape)
    except Exception:
        return False


def load_stats(model, sd):
    try:
        msd = model.state_dict()
    except Exception:
        return {"matched": 0, "mismatched": 0, "missing": None, "unexpected": None, "model_keys": None,
                "ckpt_keys": len(sd) if isinstance(sd, dict) else None, "match_ratio": None}
    matched = mismatched = 0
    for k, v in sd.items():
        if k in msd:
            if _shape_ok(msd, k, v):
                matched += 1
            else:
                mismatched += 1
    missing = len([k for k in msd if k not in sd])
    unexpected = len([k for k in sd if k not in msd])
    mk = len(msd)
    ratio = matched / float(mk) if mk else None
    return {"matched": int(matched), "mismatched": int(mismatched), "missing": int(missing),
            "unexpected": int(unexpected), "model_keys": int(mk), "ckpt_keys": int(len(sd)),
            "match_ratio": float(ratio) if ratio is not None else None}


def safe_load_state_dict(model, sd):
    msd = model.state_dict()
    filtered = {k: v for k, v in sd.items() if k in msd and _shape_ok(msd, k, v)}
    return model.load_state_dict(filtered, strict=False)


def infer_backbone_from_name(path):
    try:
        name = str(Path(path).name).lower()
    except Exception:
        return None
    for k in ("efficientnet_b0", "resnet18", "resnet34", "resnet50", "vit_base_patch16_224"):
        if k in name:
            return k
    if "efficientnet" in name:
        return "efficientnet_b0"
    if "resnet" in name:
        return "resnet50"
    if "vit" in name:
        return "vit_base_patch16_224"
    return None


def infer_single_backbone(sd):
    try:
        keys = [k for k in sd.keys() if isinstance(k, str)]
    except Exception:
        return None
    if any("backbone.patch_embed" in k or "backbone.blocks." in k for k in keys):
        return "vit_base_patch16_224"
    if any("conv_stem" in k or ".blocks." in k or "conv_dw" in k or "se.conv" in k for k in keys) and \
            any(k.startswith("backbone") for k in keys):
        return "efficientnet_b0"
    if any(".layer1." in k or ".layer2." in k or ".layer3." in k or ".layer4." in k for k in keys):
        return "resnet50"
    if any(k.startswith("backbone.0.") or k.startswith("backbone.1.") for k in keys):
        return "resnet50"
    return None


class IncompatibleCheckpoint(RuntimeError):
    pass


SUPPORTED_BACKBONES = ("efficientnet_b0", "resnet50")  # PretrainedBackboneDetector's implemented trunks


def read_checkpoint(path_or_obj, map_location="cpu"):
    if isinstance(path_or_obj, (str, Path)):
        return torch.load(str(path_or_obj), map_location=map_location, weights_only=True)
    return path_or_obj


def load_pretrained(path_or_obj, device=None, compute_dtype="fp32", checkpoint_name=None, meta=None):
    """``load_model(path, 'pretrained')`` for the HIP detector: returns ``(model, stats)`` with the
    model in eval mode on ``device``; raises ``IncompatibleCheckpoint`` where the app returns False
    (no state dict, load error, ``match_ratio < 0.80``).  ``stats`` mirrors ``LAST_LOAD_STATS``."""
    from .pretrained_detector import PretrainedBackboneDetector

    name = checkpoint_name or (str(path_or_obj) if isinstance(path_or_obj, (str, Path)) else "")
    ckpt = read_checkpoint(path_or_obj)
    sd = extract_state_dict(ckpt)
    fake_idx = detect_fake_class_index(ckpt)
    if isinstance(sd, dict) and sd:
        sd = normalize_state_dict_keys(sd)
    backbone = str((meta or {}).get("backbone") or infer_backbone_from_name(name) or "efficientnet_b0")
    if isinstance(sd, dict) and sd:
        hinted = infer_backbone_from_name(name)
        if hinted:
            backbone = hinted
        inferred = infer_single_backbone(sd)
        if inferred:
            backbone = inferred
    base = {"model_type": "pretrained"}
    if not (isinstance(sd, dict) and sd):
        raise IncompatibleCheckpoint("No state_dict found")
    if backbone not in SUPPORTED_BACKBONES:
        # app.load_model builds the timm/torchvision model and fails the match-ratio gate; the MI355X
        # path has no kernels for it: report it the same way (IncompatibleCheckpoint, with the stats)
        stats = {"backbone": backbone, "keys": len(sd), **base}
        raise IncompatibleCheckpoint(f"Unsupported backbone for the MI355X path: {backbone} "
                                     f"(supported: {', '.join(SUPPORTED_BACKBONES)}); stats={stats}")
    model = PretrainedBackboneDetector(backbone_name=backbone, pretrained=False, num_classes=2, dropout_rate=0.5,
                                       use_temporal_attention=True, compute_dtype=compute_dtype)
    stats = load_stats(model, sd)
    inc = safe_load_state_dict(model, sd)
    stats["missing"] = len(getattr(inc, "missing_keys", []) or [])
    stats["unexpected"] = len(getattr(inc, "unexpected_keys", []) or [])
    stats = {**stats, **base, "backbone": backbone, "backbones": None,
             "fake_class_index_detected": int(fake_idx) if fake_idx is not None else None}
    mr = stats.get("match_ratio")
    if mr is not None and float(mr) < 0.80:
        raise IncompatibleCheckpoint(f"Incompatible checkpoint (match_ratio={mr:.3f}).")
    if device is not None:
        model = model.to(device)
    return model.eval(), stats


def save_state_dict(model, path):
    """``EnsembleTrainer._save_checkpoint`` format: the raw state_dict (no DP prefix)."""
    torch.save(_plain_state_dict(model), str(path))


def save_training_checkpoint(path, model, optimizer=None, scheduler=None, epoch=0, metrics=None, best_f1=None):
    """``src/train.py:398-411`` format."""
    torch.save({"epoch": epoch, "model_state": _plain_state_dict(model),
                "optimizer_state": optimizer.state_dict() if optimizer is not None else None,
                "scheduler_state": scheduler.state_dict() if scheduler is not None else None,
                "metrics": metrics or {}, "best_f1": best_f1}, str(path))


def _plain_state_dict(model):
    m = getattr(model, "module", model)  # a wrapped module saves its inner keys
    return {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
