"""Fused global-norm clipping + Adam/AdamW over flat fp32 buffers (K8).

Replaces the reference step ``torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)`` +
``optimizer.step()`` with ``optim.AdamW(params, lr, weight_decay)``
(``src/ensemble_trainer.py:146,199-200``) or ``optim.Adam(params, lr)`` (``src/train.py:323``).
Update arithmetic and scalar rounding follow ``torch.optim`` (single-tensor path) so the
result matches the reference step to fp32 rounding; clipping semantics match
``clip_grad_norm_`` (coefficient ``min(1, max_norm / (norm + 1e-6))``; the gradients are left
clipped in ``.grad``).  Everything stays on the device: no ``.item()`` per step.  The parameters
are one ``FlatModule``'s (one buffer) or several (``EnsembleDetector``: one buffer per member, the
clipping norm taken over all of them, like ``clip_grad_norm_(ensemble.parameters())``).
"""
from __future__ import annotations

import torch

from . import _lib, ops  # noqa: F401  (registers torch.ops.dfd.*)


def _runs(tensors):
    """Split ``tensors`` into maximal runs of consecutive views of one storage:
    [(flat view, first index, end index)], or None if some tensor is not contiguous."""
    out, i0 = [], 0
    for i in range(1, len(tensors) + 1):
        if i < len(tensors):
            a, b = tensors[i - 1], tensors[i]
            if not b.is_contiguous():
                return None
            if (b.untyped_storage().data_ptr() == a.untyped_storage().data_ptr()
                    and b.storage_offset() == a.storage_offset() + a.numel()):
                continue
        fl = _flat_view(tensors[i0:i])
        if fl is None:
            return None
        out.append((fl, i0, i))
        i0 = i
    return out


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


class DynamicLossScaler:
    """Dynamic loss scaling for the fp16 trunk (``compute_dtype="fp16"``), the semantics of
    ``torch.amp.GradScaler(init_scale=2**16, growth_factor=2, backoff_factor=0.5,
    growth_interval=2000)`` kept entirely on the device: no ``found_inf.item()`` per step.

    State: 4 device floats ``[scale, growth tracker, found_inf, applied steps]``.  ``scale(loss)``
    multiplies the loss before backward; the fused optimizer (``FusedAdam(W).set_loss_scaler``)
    takes the norm of the scaled gradient (``found_inf`` = not finite), unscales and clips the
    gradient inside its step kernel, skips the whole step on the device when ``found_inf`` (torch
    skips ``optimizer.step()``), and then updates the scale.  Bias corrections count applied steps."""

    def __init__(self, device, init_scale: float = 2.0 ** 16, growth_factor: float = 2.0,
                 backoff_factor: float = 0.5, growth_interval: int = 2000):
        self.state = torch.tensor([float(init_scale), 0.0, 0.0, 0.0], dtype=torch.float32, device=device)
        self.growth_factor = float(growth_factor)
        self.backoff_factor = float(backoff_factor)
        self.growth_interval = int(growth_interval)

    def scale(self, loss: torch.Tensor) -> torch.Tensor:
        return loss * self.state[0]

    def update(self) -> None:
        torch.ops.dfd.loss_scale_update(self.state, self.growth_factor, self.backoff_factor, self.growth_interval)

    # host reads (synchronise; for logging / checkpoints only)
    def get_scale(self) -> float:
        return float(self.state[0])

    def applied_steps(self) -> int:
        return int(self.state[3])

    def found_inf(self) -> bool:
        return bool(self.state[2] != 0)

    def state_dict(self):
        st = self.state.cpu()
        return {"scale": float(st[0]), "_growth_tracker": int(st[1]), "growth_factor": self.growth_factor,
                "backoff_factor": self.backoff_factor, "growth_interval": self.growth_interval,
                "applied_steps": int(st[3])}

    def load_state_dict(self, sd) -> None:
        self.growth_factor = float(sd.get("growth_factor", self.growth_factor))
        self.backoff_factor = float(sd.get("backoff_factor", self.backoff_factor))
        self.growth_interval = int(sd.get("growth_interval", self.growth_interval))
        self.state.copy_(torch.tensor([float(sd["scale"]), float(sd.get("_growth_tracker", 0)), 0.0,
                                       float(sd.get("applied_steps", 0))]))


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
        self._runs = _runs(ps)
        if self._runs is None or len(self._runs) > 8:
            raise ValueError("fused Adam(W) needs the parameters of FlatModules (consecutive views of flat buffers)")
        dev = self._runs[0][0].device
        n = sum(r[0].numel() for r in self._runs)
        # run of each parameter and the moment-buffer offset of each run
        self._run_of = [0] * len(ps)
        self._run_off = []
        o = 0
        for k, (fl, i0, i1) in enumerate(self._runs):
            for i in range(i0, i1):
                self._run_of[i] = k
            self._run_off.append(o)
            o += fl.numel()
        self._m = torch.zeros(n, dtype=torch.float32, device=dev)
        self._v = torch.zeros(n, dtype=torch.float32, device=dev)
        # per-parameter step counts, as torch.optim keeps them (a parameter without a gradient is
        # skipped: no decay, no moment update, no step -- torch/optim/adamw.py semantics)
        self._steps = [0] * len(ps)
        self._offs = []
        o = 0
        for p in ps:
            self._offs.append(o)
            o += p.numel()
        self._norm = torch.zeros(2, dtype=torch.float32, device=dev)
        self._scratch = torch.empty(1024, dtype=torch.float64, device=dev)
        self.loss_scaler = None
        self._bind_state()

    def set_loss_scaler(self, scaler: "DynamicLossScaler | None") -> None:
        """Step on scaled gradients (fp16 training): see DynamicLossScaler."""
        if scaler is not None and scaler.state.device != self._m.device:
            raise ValueError("loss scaler state and optimizer state on different devices")
        self.loss_scaler = scaler
        if scaler is not None:
            with torch.no_grad():  # bias corrections continue from this optimizer's step count (resume)
                scaler.state[3] = float(self._step_count)

    def _bind_state(self):
        """``self.state[p]`` holds views of the flat moment buffers (what the kernel updates)."""
        for i, p in enumerate(self.param_groups[0]["params"]):
            o, k = self._offs[i], p.numel()
            self.state[p] = {"step": torch.tensor(float(self._steps[i])),
                             "exp_avg": self._m[o:o + k].view(p.shape), "exp_avg_sq": self._v[o:o + k].view(p.shape)}

    @property
    def _step_count(self) -> int:
        return max(self._steps) if self._steps else 0

    def _active_ranges(self):
        """[(lo, hi, first_param, last_param+1)] of consecutive parameters that have a gradient and the
        same step count (one range -- the whole buffer -- in the usual case)."""
        ps = self.param_groups[0]["params"]
        out = []
        for i, p in enumerate(ps):
            if p.grad is None or not p.requires_grad:
                continue
            lo, hi = self._offs[i], self._offs[i] + p.numel()
            if (out and out[-1][1] == lo and self._steps[out[-1][2]] == self._steps[i] and
                    self._run_of[out[-1][2]] == self._run_of[i]):
                out[-1] = (out[-1][0], hi, out[-1][2], i + 1)
            else:
                out.append((lo, hi, i, i + 1))
        return out

    def _grad_range(self, i0, i1):
        """Flat view of the gradients of parameters [i0, i1) (gathered when they are not one buffer)."""
        ps = self.param_groups[0]["params"][i0:i1]
        gs = [p.grad for p in ps]
        flat = _flat_view(gs)
        if flat is None:
            return torch.cat([g.reshape(-1) for g in gs]), gs
        return flat, None

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        g = self.param_groups[0]
        ranges = self._active_ranges()
        if not ranges:
            return loss
        grads = [self._grad_range(r[2], r[3]) for r in ranges]
        if self.loss_scaler is not None:
            return self._step_scaled(ranges, grads, loss)
        clip = None
        if self.max_grad_norm is not None:
            allg = grads[0][0] if len(grads) == 1 else torch.cat([fg for fg, _ in grads])
            torch.ops.dfd.grad_norm(allg, float(self.max_grad_norm), self._scratch, self._norm)
            clip = self._norm
        b1, b2 = g["betas"]
        for (lo, hi, i0, i1), (flat_g, scatter) in zip(ranges, grads):
            step = self._steps[i0] + 1
            for i in range(i0, i1):
                self._steps[i] = step
            k = self._run_of[i0]
            ro = self._run_off[k]
            torch.ops.dfd.adam_step(self._runs[k][0][lo - ro:hi - ro], flat_g, self._m[lo:hi], self._v[lo:hi],
                                    float(g["lr"]),
                                    float(b1), float(b2), float(g["eps"]), float(g["weight_decay"]), step,
                                    float(self.grad_scale), bool(self.decoupled), clip)
            if scatter is not None:  # gradients were gathered: leave the clipped values in .grad
                o = 0
                for t in scatter:
                    t.copy_(flat_g[o:o + t.numel()].view(t.shape))
                    o += t.numel()
        return loss

    def _step_scaled(self, ranges, grads, loss):
        """Scaled-gradient step: norm (+ found_inf) over every range, device-skipped Adam(W) per range,
        one scale update.  Several ranges arise with several flat buffers (``EnsembleDetector``: one
        per member) or frozen parameters (the reference's ``freeze_backbone``); the bias corrections
        of every range use the scaler's applied-step count (torch's per-parameter count whenever the
        trained parameters get a gradient every step, as they do in the reference's loops)."""
        sc = self.loss_scaler
        g = self.param_groups[0]
        max_norm = float(self.max_grad_norm) if self.max_grad_norm is not None else 0.0
        allg = grads[0][0] if len(grads) == 1 else torch.cat([fg for fg, _ in grads])
        torch.ops.dfd.grad_norm_scaled(allg, max_norm, sc.state, self._scratch, self._norm)
        clip = self._norm if self.max_grad_norm is not None else None
        b1, b2 = g["betas"]
        for (lo, hi, i0, i1), (flat_g, scatter) in zip(ranges, grads):
            k = self._run_of[i0]
            ro = self._run_off[k]
            torch.ops.dfd.adam_step_scaled(self._runs[k][0][lo - ro:hi - ro], flat_g, self._m[lo:hi], self._v[lo:hi],
                                           float(g["lr"]), float(b1), float(b2), float(g["eps"]),
                                           float(g["weight_decay"]), float(self.grad_scale), bool(self.decoupled),
                                           clip, sc.state)
            if scatter is not None:
                o = 0
                for t in scatter:
                    t.copy_(flat_g[o:o + t.numel()].view(t.shape))
                    o += t.numel()
        sc.update()
        self._scaled_steps = True  # per-parameter step counts live on the device (scaler applied steps)
        return loss

    # -- checkpoints: torch.optim.Adam(W)-format state ({step, exp_avg, exp_avg_sq} per parameter), so
    # a resume (src/train.py:349-387,401) works across this optimizer and torch's in both directions
    def state_dict(self):
        if getattr(self, "_scaled_steps", False) and self.loss_scaler is not None:
            n = self.loss_scaler.applied_steps()  # skipped (non-finite) steps did not count
            self._steps = [n] * len(self._steps)
        for i, p in enumerate(self.param_groups[0]["params"]):
            self.state[p]["step"] = torch.tensor(float(self._steps[i]))
        return super().state_dict()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)  # casts moments to the parameters' device/dtype
        ps = self.param_groups[0]["params"]
        with torch.no_grad():
            for i, p in enumerate(ps):
                st = self.state.get(p, {})
                o, k = self._offs[i], p.numel()
                if "exp_avg" in st:
                    self._m[o:o + k].copy_(st["exp_avg"].reshape(-1))
                    self._v[o:o + k].copy_(st["exp_avg_sq"].reshape(-1))
                    self._steps[i] = int(float(st.get("step", 0)))
                else:
                    self._m[o:o + k].zero_()
                    self._v[o:o + k].zero_()
                    self._steps[i] = 0
        self._bind_state()
        if self.loss_scaler is not None:
            with torch.no_grad():
                self.loss_scaler.state[3] = float(self._step_count)

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
    out = torch.empty(2, dtype=torch.float32, device=flat.device)
    scratch = torch.empty(1024, dtype=torch.float64, device=flat.device)
    torch.ops.dfd.grad_norm(flat, float(max_norm), scratch, out)
    for g in gs:
        g.mul_(out[1])
    return out[0]
