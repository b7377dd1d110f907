"""Flat parameter / buffer / gradient storage shared by the HIP kernels and PyTorch.

Every trainable parameter of a model lives in ONE contiguous fp32 buffer (in
``named_parameters()`` order) and each ``nn.Parameter`` is a view into it; BatchNorm
running statistics live in a second fp32 buffer and the ``num_batches_tracked`` counters in
an int64 buffer.  This gives the C ABI a single base pointer + offsets, lets the fused
optimizer and the data-parallel all-reduce work on one buffer, and keeps the reference's
``state_dict`` keys/shapes unchanged (``app.py:1413-1528`` loads by name).

Backward writes all gradients of one forward into a freshly allocated flat buffer
(``GradSink``) and hands autograd views of it; with ``p.grad is None`` autograd adopts the
view, so after ``loss.backward()`` every ``p.grad`` aliases one flat tensor.
"""
from __future__ import annotations

import torch
import torch.nn as nn


class FlatModule(nn.Module):
    """Mixin: call ``_flatten()`` after construction; ``_apply`` (``.to()``/``.cuda()``) re-packs."""

    _flat_p: torch.Tensor | None = None

    def _flatten(self) -> None:
        params = [(n, p) for n, p in self.named_parameters()]
        bufs = [(n, b) for n, b in self.named_buffers() if n.endswith(("running_mean", "running_var"))]
        cnts = [(n, b) for n, b in self.named_buffers() if n.endswith("num_batches_tracked")]
        dev = params[0][1].device if params else torch.device("cpu")
        self._p_off: dict[str, int] = {}
        self._b_off: dict[str, int] = {}
        tot = 0
        for n, p in params:
            self._p_off[n] = tot
            tot += p.numel()
        flat_p = torch.empty(tot, dtype=torch.float32, device=dev)
        tb = 0
        for n, b in bufs:
            self._b_off[n] = tb
            tb += b.numel()
        flat_b = torch.empty(max(tb, 1), dtype=torch.float32, device=dev)
        flat_c = torch.zeros(max(len(cnts), 1), dtype=torch.int64, device=dev)
        with torch.no_grad():
            for n, p in params:
                o = self._p_off[n]
                flat_p[o:o + p.numel()].copy_(p.detach().reshape(-1))
                p.data = flat_p[o:o + p.numel()].view(p.shape)
            for n, b in bufs:
                o = self._b_off[n]
                flat_b[o:o + b.numel()].copy_(b.detach().reshape(-1))
                self._set_buffer(n, flat_b[o:o + b.numel()].view(b.shape))
            for i, (n, b) in enumerate(cnts):
                flat_c[i] = b.detach().to(dev)
                self._set_buffer(n, flat_c[i:i + 1].view(()))
        self._flat_p, self._flat_b, self._flat_c = flat_p, flat_b, flat_c
        self._flat_params = params
        self._flat_bufs = bufs
        self._flat_cnts = cnts
        self._flat_ptrs = [p.data_ptr() for _, p in params] + [b.data_ptr() for _, b in bufs]
        self._on_flatten()

    def _on_flatten(self) -> None:  # subclasses bind kernels to the new offsets
        pass

    def _set_buffer(self, dotted: str, value: torch.Tensor) -> None:
        *path, leaf = dotted.split(".")
        m = self
        for q in path:
            m = getattr(m, q)
        m._buffers[leaf] = value

    def _flat_ok(self) -> bool:
        if self._flat_p is None:
            return False
        cur = [p.data_ptr() for _, p in self._flat_params] + [b.data_ptr() for _, b in self._flat_bufs]
        if cur != self._flat_ptrs:
            return False
        # a parameter replaced by a new object (load_state_dict(assign=True)) is not in our list
        return all(p is q for (_, p), (_, q) in zip(self._flat_params, self.named_parameters()))

    def ensure_flat(self) -> None:
        if not self._flat_ok():
            self._flatten()

    def _apply(self, fn, recurse=True):
        out = super()._apply(fn, recurse)
        if self._flat_p is not None:
            self._flatten()
        return out

    def param_offsets(self) -> dict[str, int]:
        return self._p_off

    def bn_offsets(self) -> dict[str, int]:
        return self._b_off


class GradSink:
    """Lazily allocated flat gradient buffer for one forward/backward of a FlatModule."""

    def __init__(self, owner: FlatModule):
        self.owner = owner
        self.flat: torch.Tensor | None = None

    def get(self) -> torch.Tensor:
        if self.flat is None:
            self.flat = torch.empty_like(self.owner._flat_p)
        return self.flat

    def views(self, names):
        g = self.get()
        out = []
        params = dict(self.owner._flat_params)
        for n in names:
            o = self.owner._p_off[n]
            p = params[n]
            out.append(g[o:o + p.numel()].view(p.shape))
        return out

    def ready(self, lo: int, hi: int) -> None:
        for h in getattr(self.owner, "_grad_ready_hooks", ()):
            h(self.get(), lo, hi)
