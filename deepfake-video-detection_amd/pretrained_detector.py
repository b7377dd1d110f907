"""Drop-in ``PretrainedBackboneDetector`` / ``EnsembleDetector`` for MI355X.

Mirrors ``src/pretrained_detector.py`` of the reference:

* ``PretrainedBackboneDetector.__init__`` (``:21-85``): same signature, attributes
  (``backbone_name``, ``num_classes``, ``feature_dim``, ``backbone``, ``temporal_attention``,
  ``dropout``, ``fc1``, ``fc2``), same head initialisation (``_init_head_weights`` ``:80-85``)
  and the same ``state_dict`` keys (``backbone.*`` = timm efficientnet_b0 names,
  ``temporal_attention.{0,2}.*``, ``fc1.*``, ``fc2.*``).
* ``forward`` (``:103-143``): ``(B, T, 3, H, W) -> (logits (B, C), frame_scores (B, T))``; the frames
  are the reference's normalised fp32 tensors, or -- new -- the raw uint8 face crops
  (``torch.from_numpy(faces).permute(0, 3, 1, 2)`` per clip) normalised inside the stem kernel
  (``input_normalization``, default the app's ImageNet constants), bit-identical to normalising
  first;
  the trunk runs as one native HIP plan, the head (temporal attention, softmax over T,
  weighted pooling, dropout, fc1/ReLU, fc2) as HIP kernels; autograd flows into every
  parameter (gradients land in one flat buffer).
* ``unfreeze_backbone`` (``:87-101``) is a no-op for EfficientNet, exactly as in the
  reference (its Sequential trunk has no ``.blocks``).

Arithmetic: ``compute_dtype="fp32"`` (default -- the drop-in meets the north-star rtol 1e-3 /
atol 1e-5 on logits and loss), ``"bf16"`` (the training/serving performance mode; bounds in
tests/test_b0_224_gpu.py and tests/test_serving.py) or ``"fp16"`` (EfficientNet-B0 only: IEEE half
storage with fp32 accumulation, trained under dynamic loss scaling by ``trainer.TrainStep``).

Backbones: ``efficientnet_b0`` (the hot path: training and inference) and ``resnet50`` (the app's
default ensemble member, ``app.py:661,1597`` -- ``resnet.ResNet50Trunk``, torchvision key names;
inference on implicit-GEMM MFMA kernels with the eval BatchNorm folded in, training in fp32 with
train-mode BatchNorm on the implicit-GEMM forward / data-gradient / weight-gradient kernels).  ``pretrained=True`` would download timm /
torchvision weights in the reference and is refused here (offline; load a checkpoint instead).
"""
from __future__ import annotations

import ctypes
from typing import List, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from .backbone import FEATURE_DIM, EfficientNetB0Trunk
from .resnet import FEATURE_DIM as RESNET_FEATURE_DIM
from .resnet import ResNet50Trunk
from .flat import FlatModule, GradSink

ATTN_HIDDEN = 64
FC1_DIM = 256


class PretrainedBackboneDetector(FlatModule):
    accepts_uint8_frames = True  # raw uint8 crops are normalised inside the stem kernel
    def __init__(self, backbone_name: str = "efficientnet_b0", pretrained: bool = True, num_classes: int = 2,
                 dropout_rate: float = 0.5, freeze_backbone: bool = False, use_temporal_attention: bool = True,
                 compute_dtype: str = "fp32", input_normalization="imagenet"):
        super().__init__()
        if backbone_name not in ("efficientnet_b0", "resnet50"):
            raise ValueError(f"Unsupported backbone: {backbone_name} (the MI355X path implements "
                             f"efficientnet_b0 and resnet50)")
        if pretrained:
            raise RuntimeError("pretrained=True fetches timm ImageNet weights, which is unavailable offline; "
                               "construct with pretrained=False and load a checkpoint (app.py:1691 does)")
        self.backbone_name = backbone_name
        self.num_classes = num_classes
        self.use_temporal_attention = use_temporal_attention
        if backbone_name == "resnet50":  # src/pretrained_detector.py:37-40 (fc.in_features = 2048)
            self.backbone = ResNet50Trunk(compute_dtype, input_normalization)
            self.feature_dim = RESNET_FEATURE_DIM
        else:
            self.backbone = EfficientNetB0Trunk(compute_dtype, input_normalization)
            self.feature_dim = FEATURE_DIM
        if freeze_backbone:
            for p in self.backbone.parameters():
                p.requires_grad = False
        if use_temporal_attention:
            self.temporal_attention = nn.Sequential(
                nn.Linear(self.feature_dim, ATTN_HIDDEN), nn.ReLU(), nn.Linear(ATTN_HIDDEN, 1), nn.Sigmoid())
        self.dropout = nn.Dropout(dropout_rate)
        self.fc1 = nn.Linear(self.feature_dim, FC1_DIM)
        self.fc2 = nn.Linear(FC1_DIM, num_classes)
        self._init_head_weights()
        self._grad_ready_hooks = []
        self._flatten()

    def _init_head_weights(self):
        nn.init.kaiming_normal_(self.fc1.weight, mode="fan_out", nonlinearity="relu")
        nn.init.constant_(self.fc1.bias, 0)
        nn.init.normal_(self.fc2.weight, 0, 0.01)
        nn.init.constant_(self.fc2.bias, 0)

    def unfreeze_backbone(self, num_blocks: int = 2):
        """pretrained_detector.py:87-101: resnet -> the last ``num_blocks`` children of the trunk;
        efficientnet -> ``backbone.blocks`` (absent on the Sequential trunk: a no-op)."""
        if self.backbone_name.startswith("resnet"):
            for layer in list(self.backbone.children())[-num_blocks:]:
                for p in layer.parameters():
                    p.requires_grad = True
        elif hasattr(self.backbone, "blocks"):
            for block in self.backbone.blocks[-num_blocks:]:
                for p in block.parameters():
                    p.requires_grad = True

    @property
    def compute_dtype(self) -> str:
        return self.backbone.compute_dtype

    @compute_dtype.setter
    def compute_dtype(self, v: str) -> None:
        self.backbone.compute_dtype = v

    def _on_flatten(self) -> None:
        if isinstance(self.backbone, EfficientNetB0Trunk):
            self.backbone.attach(self, "backbone.")
        names = self._head_param_names()
        self._head_names = names
        lo = self._p_off[names[0]]
        last = dict(self._flat_params)[names[-1]]
        self._head_range = (lo, self._p_off[names[-1]] + last.numel())

    def _head_param_names(self) -> List[str]:
        n = []
        if self.use_temporal_attention:
            n += ["temporal_attention.0.weight", "temporal_attention.0.bias",
                  "temporal_attention.2.weight", "temporal_attention.2.bias"]
        n += ["fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias"]
        return n

    def register_grad_ready_hook(self, fn):
        """``fn(flat_grad, lo, hi)`` is called (inside backward, in reverse network order) as soon as
        the gradients of flat range [lo, hi) have been enqueued -- used for bucketed all-reduce."""
        self._grad_ready_hooks.append(fn)
        return fn

    def forward(self, x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        self.ensure_flat()
        batch_size, num_frames, c, h, w = x.shape
        x_flat = x.reshape(batch_size * num_frames, c, h, w)
        sink = GradSink(self)
        if isinstance(self.backbone, ResNet50Trunk):
            feats = self.backbone(x_flat, grad_sink=sink)  # (B*T, 2048); train mode: resnet._RnTrainFn
        else:
            feats = self.backbone(x_flat, grad_sink=sink)  # (B*T, 1280)
        p = float(self.dropout.p) if self.training else 0.0
        seed = int(torch.randint(0, 2**62, (1,)).item()) if p > 0 else 0
        params = [dict(self._flat_params)[n] for n in self._head_names]
        need_grad = torch.is_grad_enabled() and (feats.requires_grad or any(q.requires_grad for q in params))
        if not need_grad:
            return _head_forward(self, feats, batch_size, num_frames, seed, p)[:2]
        return _HeadFn.apply(feats, self, sink, batch_size, num_frames, seed, p, *params)


def _head_ptrs(det: PretrainedBackboneDetector, tensors) -> ctypes.Array:
    arr = (ctypes.c_void_p * 8)()
    if det.use_temporal_attention:
        for i, t in enumerate(tensors):
            arr[i] = t.data_ptr()
    else:  # no attention MLP: fc1/fc2 occupy slots 4..7, slots 0..3 unused
        for i, t in enumerate(tensors):
            arr[4 + i] = t.data_ptr()
    return arr


def _head_forward(det, feats, B, T, seed, p):
    lib = _lib.load()
    dev = feats.device
    params = [dict(det._flat_params)[n] for n in det._head_names]
    work = torch.empty(int(lib.dfd_head_work_floats(B, T, det.feature_dim, ATTN_HIDDEN, FC1_DIM)),
                       dtype=torch.float32, device=dev)
    logits = torch.empty(B, det.num_classes, dtype=torch.float32, device=dev)
    scores = torch.empty(B, T, dtype=torch.float32, device=dev)
    _lib.check(lib.dfd_head_forward(_lib.stream_of(dev), B, T, det.feature_dim, ATTN_HIDDEN, FC1_DIM, det.num_classes,
                                    1 if det.use_temporal_attention else 0, _head_ptrs(det, params),
                                    feats.data_ptr(), work.data_ptr(), seed, p, logits.data_ptr(),
                                    scores.data_ptr()))
    return logits, scores, work


class _HeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, feats, det, sink, B, T, seed, p, *params):
        feats = feats.contiguous()
        logits, scores, work = _head_forward(det, feats, B, T, seed, p)
        ctx.det, ctx.sink, ctx.B, ctx.T, ctx.seed, ctx.p, ctx.work = det, sink, B, T, seed, p, work
        ctx.save_for_backward(feats, scores)
        if not det.use_temporal_attention:
            ctx.mark_non_differentiable(scores)
        return logits, scores

    @staticmethod
    def backward(ctx, dlogits, dscores):
        feats, scores = ctx.saved_tensors
        det = ctx.det
        lib = _lib.load()
        dev = feats.device
        if dlogits is None:
            dlogits = torch.zeros(ctx.B, det.num_classes, device=dev)
        dlogits = dlogits.contiguous().float()
        if dscores is not None:
            dscores = dscores.contiguous().float()
        dfeat = torch.empty_like(feats)
        params = [dict(det._flat_params)[n] for n in det._head_names]
        gviews = ctx.sink.views(det._head_names)
        _lib.check(lib.dfd_head_backward(_lib.stream_of(dev), ctx.B, ctx.T, det.feature_dim, ATTN_HIDDEN, FC1_DIM,
                                         det.num_classes, 1 if det.use_temporal_attention else 0,
                                         _head_ptrs(det, params), feats.data_ptr(), ctx.work.data_ptr(), ctx.seed,
                                         ctx.p, scores.data_ptr(), dlogits.data_ptr(), _lib.ptr(dscores),
                                         dfeat.data_ptr(), _head_ptrs(det, gviews)))
        ctx.sink.ready(*det._head_range)
        ctx.work = None
        return (dfeat, None, None, None, None, None, None, *gviews)


class EnsembleDetector(nn.Module):
    """``src/pretrained_detector.py:146-218``: efficientnet_b0 and resnet50 members (the app's
    default ``['efficientnet_b0', 'resnet50']``) run on the HIP path; the ensemble combination is a
    few ops on (M, B, C) logits.  Both members train (``EnsembleTrainer.train_epoch``,
    src/ensemble_trainer.py:158-229); the resnet50 member trains in fp32."""

    accepts_uint8_frames = True

    def __init__(self, backbone_names: List[str], pretrained: bool = True, num_classes: int = 2,
                 dropout_rate: float = 0.5, ensemble_method: str = "average", compute_dtype: str = "fp32"):
        super().__init__()
        self.models = nn.ModuleList([
            PretrainedBackboneDetector(backbone_name=name, pretrained=pretrained, num_classes=num_classes,
                                       dropout_rate=dropout_rate, use_temporal_attention=True,
                                       compute_dtype=compute_dtype)
            for name in backbone_names])
        self.ensemble_method = ensemble_method
        if ensemble_method == "weighted":
            self.weights = nn.Parameter(torch.ones(len(backbone_names)) / len(backbone_names))

    def forward(self, x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        outs = [m(x) for m in self.models]
        logits = torch.stack([o[0] for o in outs], dim=0)
        scores = torch.stack([o[1] for o in outs], dim=0)
        if self.ensemble_method == "average":
            return logits.mean(dim=0), scores.mean(dim=0)
        if self.ensemble_method == "weighted":
            w = F.softmax(self.weights, dim=0)
            return (logits * w.view(-1, 1, 1)).sum(dim=0), (scores * w.view(-1, 1, 1)).sum(dim=0)
        if self.ensemble_method == "voting":
            preds = logits.argmax(dim=-1)
            ens = torch.mode(preds, dim=0)[0]
            return F.one_hot(ens, num_classes=2).float(), scores.mean(dim=0)
        raise ValueError(f"Unknown ensemble method: {self.ensemble_method}")
