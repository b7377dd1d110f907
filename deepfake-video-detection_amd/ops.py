"""``torch.ops.dfd.*``: the hot-path kernels registered as PyTorch operators.

The drop-in boundary is the ``nn.Module`` contract; under it the modules call these operators, and
under the operators sits the C ABI of ``libdfd_hip.so`` (``include/dfd_hip.h``).  Registration uses
``torch.library.custom_op`` (schema, HIP implementation on the "cuda" device type, a fake/meta
implementation for shape propagation, and autograd where the op is differentiable on its own):

  dfd::b0_trunk_forward / dfd::b0_trunk_backward   the EfficientNet-B0 trunk plan (timm conv_stem ..
                                                   global_pool, src/pretrained_detector.py:116)
  dfd::weighted_cross_entropy (+ _backward)        nn.CrossEntropyLoss(weight) (ensemble_trainer.py:358)
  dfd::grad_norm, dfd::adam_step                   clip_grad_norm_(1.0) + AdamW (ensemble_trainer.py:196-200)
  dfd::grad_norm_scaled, dfd::adam_step_scaled,    the same under dynamic loss scaling (fp16 training:
  dfd::loss_scale_update                           GradScaler unscale_ / step / update, on the device)
  dfd::collate_frames                              the collate gather + /255 (train.py:38-61)

Every operator runs on the caller's current HIP stream and raises ``RuntimeError`` (``DFDError``) on
failure: there is no CPU implementation and no fallback.  The trunk operators take the plan as an
integer handle owned by the module's ``B0Runtime`` (per-model state, no process-wide cache)."""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
from torch import Tensor

from . import _lib

FEATURE_DIM = 1280
INPUT_F32, INPUT_U8 = 0, 1


def _norm_arr(norm: List[float]):
    import ctypes

    if len(norm) != 6:
        raise _lib.DFDError("input normalisation needs 3 means and 3 stds")
    return (ctypes.c_float * 6)(*[float(v) for v in norm])


def _strides(x: Tensor):
    import ctypes

    return (ctypes.c_int64 * 4)(*x.stride())


# ---------------------------------------------------------------- B0 trunk
@torch.library.custom_op("dfd::b0_trunk_forward", mutates_args=("buffers",), device_types="cuda")
def b0_trunk_forward(frames: Tensor, plan: int, params: Tensor, buffers: Tensor, norm: List[float], training: bool,
                     momentum: float) -> Tuple[Tensor, Tensor]:
    """frames (N,3,H,W) fp32 or uint8, any strides -> (features (N,1280) fp32, saved-activation workspace).
    Train mode updates the BatchNorm running statistics in ``buffers``."""
    lib = _lib.load()
    ws = torch.empty(int(lib.dfd_b0_workspace_bytes(plan)), dtype=torch.uint8, device=frames.device)
    feats = torch.empty(frames.shape[0], FEATURE_DIM, dtype=torch.float32, device=frames.device)
    fmt = INPUT_U8 if frames.dtype == torch.uint8 else INPUT_F32
    _lib.check(lib.dfd_b0_forward_ex(plan, _lib.stream_of(frames.device), frames.data_ptr(), fmt, _strides(frames),
                                     _norm_arr(norm), params.data_ptr(), buffers.data_ptr(), ws.data_ptr(),
                                     feats.data_ptr(), 1 if training else 0, float(momentum)))
    return feats, ws


@b0_trunk_forward.register_fake
def _(frames, plan, params, buffers, norm, training, momentum):
    n = int(_lib.load().dfd_b0_workspace_bytes(plan))
    return frames.new_empty(frames.shape[0], FEATURE_DIM, dtype=torch.float32), frames.new_empty(n, dtype=torch.uint8)


# workspace: the backward reuses its scratch regions (activation gradients, BN/SE partials, slabs)
@torch.library.custom_op("dfd::b0_trunk_backward", mutates_args=("workspace", "grads"), device_types="cuda")
def b0_trunk_backward(frames: Tensor, plan: int, dfeat: Tensor, params: Tensor, workspace: Tensor, grads: Tensor,
                      norm: List[float], training: bool, seg_begin: int, seg_end: int, accumulate: bool) -> None:
    """Backward of trunk segments [seg_begin, seg_end) (output side first) into the flat ``grads``."""
    lib = _lib.load()
    fmt = INPUT_U8 if frames.dtype == torch.uint8 else INPUT_F32
    dfeat = dfeat.contiguous().float()
    _lib.check(lib.dfd_b0_backward_ex(plan, _lib.stream_of(frames.device), frames.data_ptr(), fmt, _strides(frames),
                                      _norm_arr(norm), dfeat.data_ptr(), params.data_ptr(), workspace.data_ptr(),
                                      grads.data_ptr(), 1 if training else 0, int(seg_begin), int(seg_end),
                                      1 if accumulate else 0))


@b0_trunk_backward.register_fake
def _(frames, plan, dfeat, params, workspace, grads, norm, training, seg_begin, seg_end, accumulate):
    return None


# ---------------------------------------------------------------- weighted cross entropy
@torch.library.custom_op("dfd::weighted_cross_entropy", mutates_args=(), device_types="cuda")
def weighted_cross_entropy(logits: Tensor, target: Tensor, weight: Optional[Tensor],
                           ignore_index: int) -> Tuple[Tensor, Tensor]:
    """-> (mean loss (), sum of the applied class weights (1,)), nn.CrossEntropyLoss(weight, reduction='mean')."""
    lib = _lib.load()
    logits = logits.contiguous().float()
    target = target.contiguous().long()
    B, NC = logits.shape
    out = torch.empty(2, dtype=torch.float32, device=logits.device)
    _lib.check(lib.dfd_ce_forward(_lib.stream_of(logits.device), logits.data_ptr(), target.data_ptr(),
                                  _lib.ptr(weight), B, NC, ignore_index, out.data_ptr(), out[1:].data_ptr()))
    return out[0].clone(), out[1:].clone()


@weighted_cross_entropy.register_fake
def _(logits, target, weight, ignore_index):
    return logits.new_empty((), dtype=torch.float32), logits.new_empty(1, dtype=torch.float32)


@torch.library.custom_op("dfd::weighted_cross_entropy_backward", mutates_args=(), device_types="cuda")
def weighted_cross_entropy_backward(grad: Tensor, logits: Tensor, target: Tensor, weight: Optional[Tensor],
                                    ignore_index: int, wsum: Tensor) -> Tensor:
    lib = _lib.load()
    logits = logits.contiguous().float()
    target = target.contiguous().long()
    B, NC = logits.shape
    g = grad.contiguous().float().reshape(1)
    d = torch.empty_like(logits)
    _lib.check(lib.dfd_ce_backward(_lib.stream_of(logits.device), logits.data_ptr(), target.data_ptr(),
                                   _lib.ptr(weight), B, NC, ignore_index, wsum.data_ptr(), g.data_ptr(),
                                   d.data_ptr()))
    return d


@weighted_cross_entropy_backward.register_fake
def _(grad, logits, target, weight, ignore_index, wsum):
    return torch.empty_like(logits, dtype=torch.float32)


def _ce_setup(ctx, inputs, output):
    logits, target, weight, ignore_index = inputs
    ctx.save_for_backward(logits, target, output[1])
    ctx.weight, ctx.ignore_index = weight, ignore_index


def _ce_backward(ctx, gloss, _gwsum):
    logits, target, wsum = ctx.saved_tensors
    d = torch.ops.dfd.weighted_cross_entropy_backward(gloss, logits, target, ctx.weight, ctx.ignore_index, wsum)
    return d, None, None, None


weighted_cross_entropy.register_autograd(_ce_backward, setup_context=_ce_setup)


# ---------------------------------------------------------------- optimizer
# scratch: the kernel's fixed-order partial sums (written); out: [norm, clip coefficient]
@torch.library.custom_op("dfd::grad_norm", mutates_args=("scratch", "out"), device_types="cuda")
def grad_norm(grads: Tensor, max_norm: float, scratch: Tensor, out: Tensor) -> None:
    """out[0] = ||grads||_2 (fp64 accumulation, fixed order), out[1] = clip coefficient
    min(1, max_norm / (norm + 1e-6)) -- clip_grad_norm_ (torch/nn/utils/clip_grad.py)."""
    _lib.check(_lib.load().dfd_grad_norm(_lib.stream_of(grads.device), grads.data_ptr(), grads.numel(),
                                         float(max_norm), scratch.data_ptr(), out.data_ptr()))


@grad_norm.register_fake
def _(grads, max_norm, scratch, out):
    return None


# grads: with `clip` the kernel writes the clipped gradient back (FusedAdam leaves it in .grad, as
# clip_grad_norm_ does in place)
@torch.library.custom_op("dfd::adam_step", mutates_args=("params", "grads", "exp_avg", "exp_avg_sq"),
                         device_types="cuda")
def adam_step(params: Tensor, grads: Tensor, exp_avg: Tensor, exp_avg_sq: Tensor, lr: float, beta1: float,
              beta2: float, eps: float, weight_decay: float, step: int, grad_scale: float, decoupled: bool,
              clip: Optional[Tensor]) -> None:
    """One Adam (decoupled=False) / AdamW step over a flat fp32 range, with the clip coefficient of
    dfd::grad_norm applied to the gradient first (torch/optim/adamw.py semantics)."""
    _lib.check(_lib.load().dfd_adam_step(_lib.stream_of(params.device), params.data_ptr(), grads.data_ptr(),
                                         exp_avg.data_ptr(), exp_avg_sq.data_ptr(), params.numel(), float(lr),
                                         float(beta1), float(beta2), float(eps), float(weight_decay), int(step),
                                         float(grad_scale), 1 if decoupled else 0,
                                         None if clip is None else clip.data_ptr()))


@adam_step.register_fake
def _(params, grads, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay, step, grad_scale, decoupled, clip):
    return None


# dynamic loss scaling (fp16 training): `scaler` is the 4-float device state of optim.DynamicLossScaler
@torch.library.custom_op("dfd::grad_norm_scaled", mutates_args=("scaler", "scratch", "out"), device_types="cuda")
def grad_norm_scaled(grads: Tensor, max_norm: float, scaler: Tensor, scratch: Tensor, out: Tensor) -> None:
    """dfd::grad_norm of the SCALED gradient: out[0] = the unscaled norm, scaler[2] = found_inf."""
    _lib.check(_lib.load().dfd_grad_norm_scaled(_lib.stream_of(grads.device), grads.data_ptr(), grads.numel(),
                                                float(max_norm), scaler.data_ptr(), scratch.data_ptr(),
                                                out.data_ptr()))


@grad_norm_scaled.register_fake
def _(grads, max_norm, scaler, scratch, out):
    return None


@torch.library.custom_op("dfd::adam_step_scaled", mutates_args=("params", "grads", "exp_avg", "exp_avg_sq"),
                         device_types="cuda")
def adam_step_scaled(params: Tensor, grads: Tensor, exp_avg: Tensor, exp_avg_sq: Tensor, lr: float, beta1: float,
                     beta2: float, eps: float, weight_decay: float, grad_scale: float, decoupled: bool,
                     clip: Optional[Tensor], scaler: Tensor) -> None:
    """dfd::adam_step on grads / scale, skipped on device when the scaler saw a non-finite norm; the
    bias corrections count applied steps only (scaler[3])."""
    _lib.check(_lib.load().dfd_adam_step_scaled(_lib.stream_of(params.device), params.data_ptr(), grads.data_ptr(),
                                                exp_avg.data_ptr(), exp_avg_sq.data_ptr(), params.numel(), float(lr),
                                                float(beta1), float(beta2), float(eps), float(weight_decay),
                                                float(grad_scale), 1 if decoupled else 0,
                                                None if clip is None else clip.data_ptr(), scaler.data_ptr()))


@adam_step_scaled.register_fake
def _(params, grads, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay, grad_scale, decoupled, clip, scaler):
    return None


@torch.library.custom_op("dfd::loss_scale_update", mutates_args=("scaler",), device_types="cuda")
def loss_scale_update(scaler: Tensor, growth_factor: float, backoff_factor: float, growth_interval: int) -> None:
    """GradScaler.update on the device state (no host synchronisation)."""
    _lib.check(_lib.load().dfd_loss_scale_update(_lib.stream_of(scaler.device), scaler.data_ptr(),
                                                 float(growth_factor), float(backoff_factor), int(growth_interval)))


@loss_scale_update.register_fake
def _(scaler, growth_factor, backoff_factor, growth_interval):
    return None


# ---------------------------------------------------------------- input pipeline
@torch.library.custom_op("dfd::collate_frames", mutates_args=(), device_types="cuda")
def collate_frames(src: Tensor, sel: Tensor, frame_shape: List[int], to_float: bool) -> Tensor:
    """out[s] = src[sel[s]] (sel < 0: a zero frame), uint8 or fp32 v/255; src (F, *frame_shape) uint8."""
    n = sel.numel()
    fb = 1
    for d in frame_shape:
        fb *= int(d)
    out = torch.empty((n, *frame_shape), dtype=torch.float32 if to_float else torch.uint8, device=src.device)
    _lib.check(_lib.load().dfd_collate_frames(_lib.stream_of(src.device), src.data_ptr(), sel.data_ptr(), n, fb,
                                              1 if to_float else 0, out.data_ptr()))
    return out


@collate_frames.register_fake
def _(src, sel, frame_shape, to_float):
    return src.new_empty((sel.numel(), *frame_shape), dtype=torch.float32 if to_float else torch.uint8)


OPS = ("b0_trunk_forward", "b0_trunk_backward", "weighted_cross_entropy", "weighted_cross_entropy_backward",
       "grad_norm", "adam_step", "grad_norm_scaled", "adam_step_scaled", "loss_scale_update", "collate_frames")
