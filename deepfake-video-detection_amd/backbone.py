"""EfficientNet-B0 trunk on MI355X: module tree with timm's names + the HIP plan runtime.

Drop-in for the reference's ``self.backbone`` (``src/pretrained_detector.py:43-46``):
``nn.Sequential(*list(timm.create_model('efficientnet_b0').children())[:-1])``, called as
``self.backbone(x_flat)`` with ``x_flat (B*T, 3, H, W)`` and returning ``(B*T, 1280)``
(``:116``).  The parameter/buffer names, shapes and order come from the native plan's
tensor table (``dfd_b0_tensor_info``), so ``state_dict()`` keys are exactly timm's
(``backbone.0.weight``, ``backbone.2.3.1.conv_dw.weight``, ...).

The submodules are parameter holders only: the whole trunk -- stem, 16 MBConv blocks,
conv_head, BN+SiLU, global pool -- runs as ONE native launch sequence
(``dfd_b0_forward`` / ``dfd_b0_backward``).  There is no per-layer PyTorch path and no CPU
fallback.
"""
from __future__ import annotations

import ctypes
import math

import torch
import torch.nn as nn

from . import _lib, ops  # noqa: F401  (registers torch.ops.dfd.*)
from .flat import FlatModule, GradSink

BN_EPS = 1e-5
BN_MOMENTUM = 0.1
FEATURE_DIM = 1280
DTYPES = {"fp32": 0, "float32": 0, torch.float32: 0, "bf16": 1, "bfloat16": 1, torch.bfloat16: 1,
          "fp16": 2, "float16": 2, torch.float16: 2}
INPUT_F32, INPUT_U8 = 0, 1
# normalisation applied in the stem to uint8 frames: ((v / 255) - mean) / std
NORMALIZATIONS = {
    "imagenet": ((0.485, 0.456, 0.406), (0.229, 0.224, 0.225)),  # app.imagenet_normalize (app.py:1772-1780)
    "unit": ((0.0, 0.0, 0.0), (1.0, 1.0, 1.0)),                  # `.float() / 255.0` only (src/train.py:59)
}


class _Holder(nn.Module):
    """Container mirroring a timm submodule; holds parameters, never runs on its own."""

    def forward(self, *args, **kwargs):
        raise RuntimeError("EfficientNet-B0 submodules do not run standalone: the trunk executes as one "
                           "native HIP plan (call the trunk / detector instead)")


def tensor_table():
    """[(name, kind, shape)] of the native trunk, timm state_dict order."""
    lib = _lib.load()
    out = []
    buf = ctypes.create_string_buffer(256)
    kind, nd = ctypes.c_int(), ctypes.c_int()
    shp = (ctypes.c_int64 * 4)()
    for i in range(lib.dfd_b0_tensor_count()):
        _lib.check(lib.dfd_b0_tensor_info(i, buf, 256, ctypes.byref(kind), ctypes.byref(nd), shp))
        out.append((buf.value.decode(), kind.value, tuple(shp[j] for j in range(nd.value))))
    return out


def _timm_init_(name: str, t: torch.Tensor) -> None:
    """timm ``_init_weight_goog``-style init: conv N(0, sqrt(2/fan_out)), BN 1/0, biases 0."""
    leaf = name.rsplit(".", 1)[-1]
    with torch.no_grad():
        if leaf == "weight" and t.dim() == 4:
            k = t.shape[2] * t.shape[3]
            groups = t.shape[0] if t.shape[1] == 1 and k > 1 else 1
            fan_out = k * t.shape[0] // groups
            t.normal_(0.0, math.sqrt(2.0 / fan_out))
        elif leaf == "weight":
            t.fill_(1.0)
        elif leaf in ("bias", "running_mean"):
            t.zero_()
        elif leaf == "running_var":
            t.fill_(1.0)


class EfficientNetB0Trunk(FlatModule):
    accepts_uint8_frames = True  # raw uint8 crops are normalised inside the stem kernel
    """The 6-child trunk Sequential (conv_stem, bn1, blocks, conv_head, bn2, global_pool).

    Args:
        compute_dtype: activation storage / MFMA dtype of the trunk: ``"fp32"`` (default: exact
            fp32 MFMA, the reference's arithmetic within the north-star tolerance), ``"bf16"``
            (fp32 accumulation, fp32 master weights and BN statistics; the training/serving
            performance mode, bound tested in tests/test_b0_224_gpu.py and tests/test_serving.py) or
            ``"fp16"`` (IEEE half storage on v_mfma_f32_16x16x32_f16, fp32 accumulation / master
            weights / statistics; train it with loss scaling -- TrainStep does, DynamicLossScaler).
        input_normalization: how uint8 frames are normalised inside the stem (``"imagenet"``
            as app.py:2084-2085, ``"unit"`` = /255 only as src/train.py:59, or ``(mean3, std3)``).
            fp32 frames are used as given.
    """

    def __init__(self, compute_dtype="fp32", input_normalization="imagenet"):
        super().__init__()
        self.compute_dtype = compute_dtype
        self.input_normalization = input_normalization
        self._table = tensor_table()
        for name, kind, shape in self._table:
            *path, leaf = name.split(".")
            m = self
            for q in path:
                if q not in m._modules:
                    m.add_module(q, _Holder())
                m = m._modules[q]
            if kind == 0:
                p = nn.Parameter(torch.empty(shape))
                _timm_init_(name, p)
                m.register_parameter(leaf, p)
            elif kind == 1:
                b = torch.empty(shape)
                _timm_init_(name, b)
                m.register_buffer(leaf, b)
            else:
                m.register_buffer(leaf, torch.tensor(0, dtype=torch.long))
        self.add_module("5", _Holder())  # global_pool (no parameters)
        self._runtime = None
        self._owner_ref = None
        self._prefix = ""

    # -- Sequential-like access (reference code indexes / iterates the trunk)
    def __getitem__(self, i):
        return list(self._modules.values())[i]

    def __len__(self):
        return len(self._modules)

    def __iter__(self):
        return iter(self._modules.values())

    def _owner(self) -> FlatModule:
        o = self._owner_ref() if self._owner_ref is not None else None
        return o if o is not None else self

    def attach(self, owner: FlatModule, prefix: str) -> None:
        """Called by an owning FlatModule after it flattened (this trunk's tensors live in its buffers)."""
        import weakref

        self._flat_p = None  # storage now belongs to the owner
        self._owner_ref = weakref.ref(owner)
        self._prefix = prefix
        self._bind()

    def _on_flatten(self) -> None:
        self._owner_ref = None
        self._prefix = ""
        self._bind()

    def _bind(self) -> None:
        owner = self._owner()
        po, bo = owner.param_offsets(), owner.bn_offsets()
        offs = []
        for name, kind, _ in self._table:
            full = self._prefix + name
            offs.append(po[full] if kind == 0 else (bo[full] if kind == 1 else 0))
        self._offsets = offs
        if self._runtime is not None:
            self._runtime.rebind(offs)
        # gradient segments -> flat ranges (tensor index range -> parameter offsets)
        lib = _lib.load()
        numel = {n: math.prod(shape) for n, _, shape in self._table}
        self._seg_ranges = []
        lo, hi = ctypes.c_int(), ctypes.c_int()
        for s in range(lib.dfd_b0_segment_count()):
            _lib.check(lib.dfd_b0_segment_tensors(s, ctypes.byref(lo), ctypes.byref(hi)))
            names = [n for n, k, _ in self._table[lo.value:hi.value] if k == 0]
            if names:
                a = po[self._prefix + names[0]]
                b = po[self._prefix + names[-1]] + numel[names[-1]]
                self._seg_ranges.append((a, b))
            else:
                self._seg_ranges.append((0, 0))
        self._param_names = [self._prefix + n for n, k, _ in self._table if k == 0]

    def runtime(self):
        if self._runtime is None:
            self._runtime = B0Runtime(self._offsets)
        return self._runtime

    def forward(self, x: torch.Tensor, grad_sink: GradSink | None = None) -> torch.Tensor:
        owner = self._owner()
        owner.ensure_flat()
        _lib.require_hip(x, "frames")
        if x.dim() != 4 or x.shape[1] != 3:
            raise ValueError(f"expected (N, 3, H, W) frames, got {tuple(x.shape)}")
        if x.dtype != torch.float32 and x.dtype != torch.uint8:
            x = x.float()
        if owner._flat_p.device != x.device:
            raise RuntimeError(f"frames on {x.device} but weights on {owner._flat_p.device}")
        training = self.training
        if training:
            with torch.no_grad():
                owner._flat_c.add_(1)  # BatchNorm2d num_batches_tracked (all layers at once)
        params = [p for n, p in owner._flat_params if n in self._param_name_set()]
        need_grad = torch.is_grad_enabled() and any(p.requires_grad for p in params)
        if need_grad and x.requires_grad:
            raise NotImplementedError("gradient w.r.t. the input frames is not provided by the HIP trunk")
        dt = DTYPES[self.compute_dtype]
        if x.dtype == torch.uint8:
            self.runtime().set_input_norm(self.input_normalization)
        if not need_grad:
            feats, _ = self.runtime().forward(x, owner, dt, training)
            return feats
        sink = grad_sink if grad_sink is not None else GradSink(owner)
        return _TrunkFn.apply(x, self, sink, dt, training, *params)

    def _param_name_set(self):
        s = getattr(self, "_pns", None)
        if s is None or len(s) != len(self._param_names):
            s = set(self._param_names)
            self._pns = s
        return s


# Kernel-selection overrides every NEW B0Runtime starts from (Python-side configuration, read once at
# runtime construction; the native plans hold their own copies, nothing process-wide is consulted on
# the enqueue path).  Tests and A/B tools set it before building a model, or call set_tuning on a
# model's runtime.
DEFAULT_TUNING: dict = {}


class B0Runtime:
    """Per-model plan cache: one native plan per (frames, H, W, dtype, device).

    Thread-safe: the cache is guarded by a lock (inference may run on a ThreadPoolExecutor worker,
    app.py:127-129,234, next to other callers), and the native plan serialises the enqueue of
    concurrent calls itself.  Kernel-selection knobs set through ``set_tuning`` belong to this
    runtime's plans only (``dfd_b0_plan_set_tuning``); no process-wide state is touched."""

    def __init__(self, offsets):
        import threading

        self.lib = _lib.load()
        self.offsets = list(offsets)
        self.plans: dict = {}
        self.tuning: dict = dict(DEFAULT_TUNING)
        self._lock = threading.Lock()
        self._norm = [*NORMALIZATIONS["imagenet"][0], *NORMALIZATIONS["imagenet"][1]]

    def set_input_norm(self, spec) -> None:
        mean, std = NORMALIZATIONS[spec] if isinstance(spec, str) else spec
        if len(mean) != 3 or len(std) != 3:
            raise ValueError("input normalisation needs 3 means and 3 stds")
        self._norm = [*[float(v) for v in mean], *[float(v) for v in std]]

    def set_tuning(self, key: str, value: int) -> None:
        """Per-runtime kernel-selection override (keys of dfd_b0_plan_set_tuning)."""
        with self._lock:
            self.tuning[key] = int(value)
            for h in self.plans.values():
                _lib.check(self.lib.dfd_b0_plan_set_tuning(h, key.encode(), int(value)))

    def rebind(self, offsets):
        with self._lock:
            self.offsets = list(offsets)
            arr = (ctypes.c_int64 * len(self.offsets))(*self.offsets)
            for h in self.plans.values():
                _lib.check(self.lib.dfd_b0_bind(h, arr, len(self.offsets)))

    def plan(self, frames, H, W, dtype, device):
        key = (frames, H, W, dtype, device.index)
        with self._lock:
            h = self.plans.get(key)
            if h is None:
                h = ctypes.c_void_p()
                with torch.cuda.device(device):
                    _lib.check(self.lib.dfd_b0_plan_create(frames, H, W, dtype, ctypes.byref(h)))
                    arr = (ctypes.c_int64 * len(self.offsets))(*self.offsets)
                    _lib.check(self.lib.dfd_b0_bind(h, arr, len(self.offsets)))
                    for k, v in self.tuning.items():
                        _lib.check(self.lib.dfd_b0_plan_set_tuning(h, k.encode(), v))
                self.plans[key] = h
            return h

    def workspace_bytes(self, h) -> int:
        return int(self.lib.dfd_b0_workspace_bytes(h))

    def forward(self, x, owner, dtype, training):
        """torch.ops.dfd.b0_trunk_forward on this runtime's plan for x's shape."""
        N, _, H, W = x.shape
        h = self.plan(N, H, W, dtype, x.device)
        feats, ws = torch.ops.dfd.b0_trunk_forward(x, h.value, owner._flat_p, owner._flat_b, self._norm, training,
                                                   BN_MOMENTUM)
        if training and self.tuning.get("mbconv7"):  # the eval-mode fused launch has no grid barrier
            self._check_fused_abort(h, ws)
        return feats, (h, ws)

    def _check_fused_abort(self, h, ws) -> None:
        """The experimental fused 7x7 MBConv (knob mbconv7, off by default) synchronises its grid with
        software barriers; one that times out (a grid that was not co-resident) sets an abort word and
        leaves wrong statistics.  With the knob on, every forward reads that word (one device sync)
        and raises instead of returning a silently wrong step."""
        nb, off = ctypes.c_int(), ctypes.c_int64()
        _lib.check(self.lib.dfd_b0_fused_info(h, ctypes.byref(nb), ctypes.byref(off)))
        if nb.value and int(ws[off.value:off.value + 4].view(torch.int32).item()) != 0:
            raise _lib.DFDError("fused 7x7 MBConv: a grid barrier timed out (grid not co-resident); "
                                "this step's statistics are invalid -- turn the mbconv7 knob off")

    def check_status(self, synchronize: bool = True) -> None:
        """Raise if a device-side software barrier of any of this runtime's plans timed out (the split
        SE excitation's slice sync, when another stream's kernels held the CUs its grid needed): that
        call's outputs were invalid.  The plans also refuse every later call on their own (the status
        is sticky, set by the device in pinned host memory); this is the definitive check after a
        device synchronisation (trainers call it at epoch ends, tests after a step)."""
        if synchronize:
            torch.cuda.synchronize()
        st = ctypes.c_int()
        with self._lock:
            for h in self.plans.values():
                _lib.check(self.lib.dfd_b0_plan_status(h, ctypes.byref(st)))
                if st.value:
                    raise _lib.DFDError("b0 plan: a software barrier (SE slice sync) timed out -- that step's "
                                        "outputs were invalid; call clear_status() to run the plan again")

    def clear_status(self) -> None:
        with self._lock:
            for h in self.plans.values():
                _lib.check(self.lib.dfd_b0_plan_clear_status(h))

    def backward(self, h, ws, x, dfeat, owner, grads, training, seg_begin, seg_end, accumulate=False):
        torch.ops.dfd.b0_trunk_backward(x, h.value, dfeat, owner._flat_p, ws, grads, self._norm, training, seg_begin,
                                        seg_end, accumulate)

    def __del__(self):
        try:
            for h in self.plans.values():
                self.lib.dfd_b0_plan_destroy(h)
        except Exception:
            pass


class _TrunkFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, trunk, sink, dtype, training, *params):
        owner = trunk._owner()
        feats, (h, ws) = trunk.runtime().forward(x, owner, dtype, training)
        ctx.trunk, ctx.sink, ctx.h, ctx.ws, ctx.training = trunk, sink, h, ws, training
        ctx.save_for_backward(x)
        return feats

    @staticmethod
    def backward(ctx, dfeat):
        (x,) = ctx.saved_tensors
        trunk = ctx.trunk
        owner = trunk._owner()
        grads = ctx.sink.get()
        dfeat = dfeat.contiguous().float()
        rt = trunk.runtime()
        nseg = len(trunk._seg_ranges)
        if getattr(owner, "_grad_ready_hooks", ()):
            # segment by segment: each segment's gradients are final when its call returns, so the
            # hooks (the data-parallel all-reduce buckets) can start while the rest of backward runs
            for s in range(nseg):
                rt.backward(ctx.h, ctx.ws, x, dfeat, owner, grads, ctx.training, s, s + 1)
                lo, hi = trunk._seg_ranges[s]
                if hi > lo:
                    ctx.sink.ready(lo, hi)
        else:
            # nobody waits for a segment: one call, the weight-gradient slab reductions and SE weight
            # gradients batched across segments (fewer launches)
            rt.backward(ctx.h, ctx.ws, x, dfeat, owner, grads, ctx.training, 0, nseg)
        ctx.ws = None
        views = ctx.sink.views(trunk._param_names)
        return (None, None, None, None, None, *views)


class B0FrameExtractor(EfficientNetB0Trunk):
    """Frame feature extractor for the ``DeepfakeDetector(model_type='rnn')`` seam
    (``src/detector.py:88-100``): ``(N, 3, H, W)`` face crops -> ``(N, 1280)`` pooled B0 features,
    feeding a ``LogicRNNLSTM(input_size=1280)``.  A standalone trunk owning its flat buffers.
    uint8 crops are normalised as the detector does (``/255`` only, ``detector.py:59-60``)."""

    def __init__(self, compute_dtype="fp32", input_normalization="unit"):
        super().__init__(compute_dtype, input_normalization)
