"""Weighted cross entropy on HIP -- drop-in for ``nn.CrossEntropyLoss(weight=...)``.

Reference uses: ``criterion = nn.CrossEntropyLoss(weight=class_weights)``
(``src/ensemble_trainer.py:358``, ``src/train.py:337``) on ``(B, 2)`` logits, mean reduction:
``sum_b w[y_b] * (-log softmax(z_b)[y_b]) / sum_b w[y_b]``.  Forward and backward are one HIP
kernel each (``torch.ops.dfd.weighted_cross_entropy``, autograd registered on the op) and never
synchronise with the host.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib, ops  # noqa: F401  (registers torch.ops.dfd.*)


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
        loss, _ = torch.ops.dfd.weighted_cross_entropy(logits, target, w, self.ignore_index)
        return loss
