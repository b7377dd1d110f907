"""Train-step API: the reference's ``EnsembleTrainer.train_epoch`` step on HIP, single- and multi-GPU.

Reference step (``src/ensemble_trainer.py:182-203``)::

    optimizer.zero_grad(); outputs = model(images); loss = criterion(outputs, labels)
    loss.backward(); clip_grad_norm_(model.parameters(), 1.0); optimizer.step(); loss.item()

``TrainStep`` runs exactly that with the HIP detector, the HIP weighted cross entropy and the
fused clip+AdamW kernel, without the per-step host sync (``loss.item()`` is left to the
caller).  ``DataParallelTrainer`` shards clips across ranks (one process per GPU,
``torch.distributed`` / RCCL over xGMI): gradients are summed by bucketed async all-reduce
launched from inside backward as soon as a segment's gradients are enqueued (reverse network
order: head, conv_head, stage 6, 5, ...), so communication overlaps the remaining backward
(RCCL runs on its own stream); the loss is pre-divided by the world size so the sum is the
mean.  BatchNorm statistics stay local per rank (the reference has no SyncBN).

With the fp16 trunk (``compute_dtype="fp16"``) the step scales the loss by a ``DynamicLossScaler``
before backward (fp16 activation gradients would underflow) and the fused optimizer unscales, skips
non-finite steps and updates the scale on the device (``torch.amp.GradScaler`` semantics, no sync).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .losses import WeightedCrossEntropyLoss
from .optim import DynamicLossScaler, FusedAdam, FusedAdamW


class TrainStep:
    def __init__(self, model, lr=1e-4, weight_decay=1e-5, class_weights=None, max_grad_norm=1.0,
                 optimizer="adamw", world_size: int = 1, criterion=None, loss_scale="auto"):
        self.model = model
        # the reference trainers hand the criterion in (ensemble_trainer.py:358 -> train_epoch); default:
        # the HIP weighted cross entropy
        self.criterion = criterion if criterion is not None else WeightedCrossEntropyLoss(weight=class_weights)
        cls = FusedAdamW if optimizer == "adamw" else FusedAdam
        self.optimizer = cls(model.parameters(), lr=lr, weight_decay=weight_decay, max_grad_norm=max_grad_norm)
        self.world_size = world_size
        # fp16 trunk: dynamic loss scaling (torch.amp.GradScaler semantics, on the device).  "auto" =
        # on when any submodule computes in fp16 (the detector, or a member of EnsembleDetector), off
        # otherwise; or a DynamicLossScaler / None.
        if loss_scale == "auto":
            fp16 = any(getattr(m, "compute_dtype", None) == "fp16" for m in model.modules())
            loss_scale = DynamicLossScaler(self.optimizer._m.device) if fp16 else None
        self.loss_scaler = loss_scale
        self.optimizer.set_loss_scaler(loss_scale)

    def forward_backward(self, images, labels):
        self.optimizer.zero_grad(set_to_none=True)
        out = self.model(images)
        logits = out[0] if isinstance(out, tuple) else out
        loss = self.criterion(logits, labels)
        l = loss / self.world_size if self.world_size > 1 else loss
        (self.loss_scaler.scale(l) if self.loss_scaler is not None else l).backward()
        return loss, logits

    def __call__(self, images, labels):
        loss, logits = self.forward_backward(images, labels)
        self.sync_grads()
        self.optimizer.step()
        return loss, logits

    def sync_grads(self):
        pass


class DataParallelTrainer(TrainStep):
    """One rank per GPU; bucketed RCCL all-reduce of the flat gradient overlapped with backward."""

    def __init__(self, model, bucket_elems: int = 1 << 20, process_group=None, **kw):
        ws = dist.get_world_size(process_group) if dist.is_initialized() else 1
        super().__init__(model, world_size=ws, **kw)
        self.pg = process_group
        self.bucket_elems = bucket_elems
        self._works = []
        self._pending = None  # (lo, hi) accumulated but not yet launched
        self._flat = None
        self.comm_enabled = True  # False: skip the exchange (bench's comm-off timing pass only)
        self.bucket_log = []  # (lo, hi) of the buckets launched by the last backward
        if ws > 1:
            self._broadcast_params()
            model.register_grad_ready_hook(self._on_ready)

    def _broadcast_params(self):
        with torch.no_grad():
            dist.broadcast(self.model._flat_p, src=0, group=self.pg)
            dist.broadcast(self.model._flat_b, src=0, group=self.pg)

    def _launch(self, flat, lo, hi):
        self.bucket_log.append((lo, hi))
        self._works.append(dist.all_reduce(flat[lo:hi], op=dist.ReduceOp.SUM, group=self.pg, async_op=True))

    def _check_adoption(self):
        """The buckets are all-reduced in the GradSink buffer while backward runs; that is only the
        gradient if autograd ADOPTS the sink views as ``p.grad``, i.e. every ``p.grad`` is None when
        backward starts.  An existing ``.grad`` (``zero_grad(set_to_none=False)``, gradient
        accumulation) would be added to the unreduced view instead -- refuse that loudly."""
        stale = [n for n, p in self.model.named_parameters() if p.requires_grad and p.grad is not None]
        if stale:
            raise RuntimeError(
                f"DataParallelTrainer: {len(stale)} parameters (e.g. {stale[0]}) already hold a .grad at backward; "
                "the overlapped all-reduce needs zero_grad(set_to_none=True) before every backward "
                "(gradient accumulation is not supported)")

    def _on_ready(self, flat, lo, hi):
        # segments arrive in reverse order of the flat layout: merge adjacent ranges into buckets
        if not self.comm_enabled:
            return
        if self._pending is None and not self._works:  # first segment of this backward
            self._check_adoption()
            self.bucket_log = []
        self._flat = flat
        if self._pending is None:
            self._pending = (lo, hi)
        elif hi == self._pending[0]:
            self._pending = (lo, self._pending[1])
        else:
            self._launch(flat, *self._pending)
            self._pending = (lo, hi)
        if self._pending[1] - self._pending[0] >= self.bucket_elems:
            self._launch(flat, *self._pending)
            self._pending = None

    def sync_grads(self):
        if self.world_size <= 1 or not self.comm_enabled:
            return
        if self._pending is not None:
            self._launch(self._flat, *self._pending)
            self._pending = None
        for w in self._works:
            w.wait()
        self._works.clear()
