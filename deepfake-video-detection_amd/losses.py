"""Weighted cross entropy on HIP -- drop-in for ``nn.CrossEntropyLoss(weight=...)``.

Reference uses: ``criterion = nn.CrossEntropyLoss(weight=class_weights)``
(``src/ensemble_trainer.py:358``, ``src/train.py:337``) on ``(B, 2)`` logits, mean reduction:
``sum_b w[y_b] * (-log softmax(z_b)[y_b]) / sum_b w[y_b]``.  Forward and backward are one HIP
kernel each and never synchronise with the host.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib


class _CEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, weight, ignore_index):
        lib = _lib.load()
        logits = logits.contiguous().float()
        target = target.contiguous().long()
        B, NC = logits.shape
        dev = logits.device
        out = torch.empty(2, dtype=torch.float32, device=dev)  # [loss, sum of weights]
        _lib.check(lib.dfd_ce_forward(_lib.stream_of(dev), logits.data_ptr(), target.data_ptr(), _lib.ptr(weight), B,
                                      NC, ignore_index, out.data_ptr(), out[1:].data_ptr()))
        ctx.save_for_backward(logits, target, out)
        ctx.weight, ctx.ignore_index = weight, ignore_index
        return out[0]

    @staticmethod
    def backward(ctx, gout):
        logits, target, out = ctx.saved_tensors
        lib = _lib.load()
        B, NC = logits.shape
        g = gout.contiguous().float().reshape(1)
        d = torch.empty_like(logits)
        _lib.check(lib.dfd_ce_backward(_lib.stream_of(logits.device), logits.data_ptr(), target.data_ptr(),
                                       _lib.ptr(ctx.weight), B, NC, ctx.ignore_index, out[1:].data_ptr(), g.data_ptr(),
                                       d.data_ptr()))
        return d, None, None, None


class WeightedCrossEntropyLoss(nn.Module):
    def __init__(self, weight: torch.Tensor | None = None, ignore_index: int = -100, reduction: str = "mean"):
        super().__init__()
        if reduction != "mean":
            raise NotImplementedError("only reduction='mean' (the reference's setting) is implemented")
        self.register_buffer("weight", None if weight is None else weight.detach().float().clone())
        self.ignore_index = ignore_index

    def forward(self, logits: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        _lib.require_hip(logits, "logits")
        if self.weight is not None and (self.weight.device != logits.device or not self.weight.is_contiguous()):
            # moved once: a per-step host->device copy of a pageable tensor blocks the host until the
            # queue drains (measured 7 ms/step of host stall in the bench step, tools/host_prof.py)
            self.weight = self.weight.to(logits.device).contiguous()
        w = self.weight
        return _CEFn.apply(logits, target, w, self.ignore_index)
