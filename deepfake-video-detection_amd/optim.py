"""Fused global-norm clipping + Adam/AdamW over one flat fp32 buffer (K8).

Replaces the reference step ``torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)`` +
``optimizer.step()`` with ``optim.AdamW(params, lr, weight_decay)``
(``src/ensemble_trainer.py:146,199-200``) or ``optim.Adam(params, lr)`` (``src/train.py:323``).
Update arithmetic and scalar rounding follow ``torch.optim`` (single-tensor path) so the
result matches the reference step to fp32 rounding; clipping semantics match
``clip_grad_norm_`` (coefficient ``min(1, max_norm / (norm + 1e-6))``; the gradients are left
clipped in ``.grad``).  Everything stays on the device: no ``.item()`` per step.
"""
from __future__ import annotations

import torch

from . import _lib


def _flat_view(tensors):
    """If ``tensors`` are consecutive views of one storage, return that flat range, else None."""
    t0 = tensors[0]
    st = t0.untyped_storage()
    off = t0.storage_offset()
    for t in tensors:
        if t.untyped_storage().data_ptr() != st.data_ptr() or t.storage_offset() != off or not t.is_contiguous():
            return None
        off += t.numel()
    flat = torch.empty(0, dtype=t0.dtype, device=t0.device)
    flat.set_(st, t0.storage_offset(), (off - t0.storage_offset(),))
    return flat


class _FusedAdamBase(torch.optim.Optimizer):
    decoupled = True

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, max_grad_norm=None,
                 grad_scale=1.0):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        if len(self.param_groups) != 1:
            raise ValueError("fused Adam(W) supports a single parameter group")
        self.max_grad_norm = max_grad_norm
        self.grad_scale = grad_scale
        ps = self.param_groups[0]["params"]
        self._flat_p = _flat_view(ps)
        if self._flat_p is None:
            raise ValueError("fused Adam(W) needs the parameters of one FlatModule (consecutive views of one buffer)")
        dev = self._flat_p.device
        n = self._flat_p.numel()
        self._m = torch.zeros(n, dtype=torch.float32, device=dev)
        self._v = torch.zeros(n, dtype=torch.float32, device=dev)
        self._step_count = 0
        self._norm = torch.zeros(2, dtype=torch.float32, device=dev)
        self._scratch = torch.empty(1024, dtype=torch.float64, device=dev)
        o = 0
        for p in ps:
            k = p.numel()
            self.state[p] = {"exp_avg": self._m[o:o + k].view(p.shape), "exp_avg_sq": self._v[o:o + k].view(p.shape)}
            o += k

    def _flat_grad(self):
        ps = self.param_groups[0]["params"]
        gs = [p.grad for p in ps]
        if any(g is None for g in gs):
            gs = [torch.zeros_like(p) if p.grad is None else p.grad for p in ps]
            for p, g in zip(ps, gs):
                p.grad = g
        flat = _flat_view(gs)
        if flat is None:  # gradients not adopted from one flat sink: gather once, scatter back below
            flat = torch.cat([g.reshape(-1) for g in gs])
            return flat, gs
        return flat, None

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        g = self.param_groups[0]
        lib = _lib.load()
        flat_g, scatter = self._flat_grad()
        dev = flat_g.device
        stream = _lib.stream_of(dev)
        n = flat_g.numel()
        clip = None
        if self.max_grad_norm is not None:
            _lib.check(lib.dfd_grad_norm(stream, flat_g.data_ptr(), n, float(self.max_grad_norm),
                                         self._scratch.data_ptr(), self._norm.data_ptr()))
            clip = self._norm.data_ptr()
        self._step_count += 1
        b1, b2 = g["betas"]
        _lib.check(lib.dfd_adam_step(stream, self._flat_p.data_ptr(), flat_g.data_ptr(), self._m.data_ptr(),
                                     self._v.data_ptr(), n, float(g["lr"]), float(b1), float(b2), float(g["eps"]),
                                     float(g["weight_decay"]), self._step_count, float(self.grad_scale),
                                     1 if self.decoupled else 0, clip))
        if scatter is not None:
            o = 0
            for t in scatter:
                t.copy_(flat_g[o:o + t.numel()].view(t.shape))
                o += t.numel()
        return loss

    @property
    def last_grad_norm(self) -> torch.Tensor:
        """Device tensor with the total gradient norm of the last step (no sync)."""
        return self._norm[0]


class FusedAdamW(_FusedAdamBase):
    """``torch.optim.AdamW`` (+ optional fused ``clip_grad_norm_``) on the flat buffer."""

    decoupled = True

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, max_grad_norm=None,
                 grad_scale=1.0):
        super().__init__(params, lr, betas, eps, weight_decay, max_grad_norm, grad_scale)


class FusedAdam(_FusedAdamBase):
    """``torch.optim.Adam`` (L2 penalty folded into the gradient) on the flat buffer."""

    decoupled = False

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, max_grad_norm=None,
                 grad_scale=1.0):
        super().__init__(params, lr, betas, eps, weight_decay, max_grad_norm, grad_scale)


def clip_grad_norm_(parameters, max_norm: float) -> torch.Tensor:
    """HIP ``torch.nn.utils.clip_grad_norm_`` for flat-buffer gradients; returns the total norm (device)."""
    ps = [p for p in parameters if p.grad is not None]
    gs = [p.grad for p in ps]
    flat = _flat_view(gs)
    if flat is None:
        flat = torch.cat([g.reshape(-1) for g in gs])
    lib = _lib.load()
    out = torch.empty(2, dtype=torch.float32, device=flat.device)
    scratch = torch.empty(1024, dtype=torch.float64, device=flat.device)
    _lib.check(lib.dfd_grad_norm(_lib.stream_of(flat.device), flat.data_ptr(), flat.numel(), float(max_norm),
                                 scratch.data_ptr(), out.data_ptr()))
    for g in gs:
        g.mul_(out[1])
    return out[0]
