"""ResNet-50 ensemble member on MI355X: ``PretrainedBackboneDetector(backbone_name='resnet50')``.

Reference: ``src/pretrained_detector.py:37-40`` builds ``torchvision.models.resnet50`` and keeps
``nn.Sequential(*children()[:-1])`` (feature_dim 2048); ``EnsembleDetector`` (``:146-218``) pairs
it with EfficientNet-B0 in the app's default ensemble (``ENSEMBLE_BACKBONES``, ``app.py:661,1597``),
which serving runs in eval mode (``app.load_model`` -> ``model.eval()``, ``predict_video``).

``ResNet50Trunk`` keeps torchvision's module tree (so ``state_dict`` keys are ``0.weight`` (conv1),
``1.*`` (bn1), ``4.0.conv1.weight`` ... under the detector's ``backbone.`` prefix) and runs the
INFERENCE forward on HIP, NHWC:

* every convolution is ``dfd_rn_conv``, an implicit-GEMM MFMA kernel (``csrc/k_rnconv.hip``: the
  im2col rows are gathered inside the A-tile staging, never materialised; fp32 accumulation) with
  the eval-mode BatchNorm folded into the weights and a bias; ReLU and the bottleneck's identity
  add run in its epilogue: ``relu(conv3(x) * s3 + b3 + identity)``.  No library GEMM;
* conv1 (Cin = 3) reads the (N,3,H,W) frames through ``dfd_rn_stem_im2col`` (any strides, fp32 or
  uint8 with the input normalisation inside, like the B0 stem) and runs on the same MFMA kernel
  (``dfd_rn_gemm``); maxpool and the global average pool are HIP kernels (``csrc/k_resnet.hip``).

Training mode is not provided for this member (the hot path trains EfficientNet-B0): calling it
with gradients enabled, or in ``.train()`` mode, raises instead of silently using batch statistics.
"""
from __future__ import annotations

import ctypes
from typing import List

import torch
import torch.nn as nn

from . import _lib

LAYERS = (3, 4, 6, 3)
PLANES = (64, 128, 256, 512)
EXPANSION = 4
FEATURE_DIM = 2048
BN_EPS = 1e-5
STEM_KP = 152  # conv1 im2col row: 7*7*3 = 147 taps + zero padding to a 16-B multiple
DTYPES = {"fp32": 0, "bf16": 1}
TORCH_DT = {0: torch.float32, 1: torch.bfloat16}


class Bottleneck(nn.Module):
    """torchvision ``Bottleneck`` (v1.5: the stride sits on conv2): parameters and names only."""

    expansion = EXPANSION

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * EXPANSION, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * EXPANSION)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride


def _make_layer(inplanes, planes, blocks, stride):
    downsample = None
    if stride != 1 or inplanes != planes * EXPANSION:
        downsample = nn.Sequential(nn.Conv2d(inplanes, planes * EXPANSION, 1, stride=stride, bias=False),
                                   nn.BatchNorm2d(planes * EXPANSION))
    layers = [Bottleneck(inplanes, planes, stride, downsample)]
    for _ in range(1, blocks):
        layers.append(Bottleneck(planes * EXPANSION, planes))
    return nn.Sequential(*layers)


def _torchvision_init_(m: nn.Module) -> None:
    """torchvision ResNet.__init__: kaiming_normal_(fan_out, relu) convs, BN weight 1 / bias 0."""
    for mod in m.modules():
        if isinstance(mod, nn.Conv2d):
            nn.init.kaiming_normal_(mod.weight, mode="fan_out", nonlinearity="relu")
        elif isinstance(mod, nn.BatchNorm2d):
            nn.init.constant_(mod.weight, 1)
            nn.init.constant_(mod.bias, 0)


class _Conv:
    """One folded convolution: packed weights [Cout][kh*kw*Cin (+pad)] in the compute dtype + fp32 bias."""

    __slots__ = ("w", "b", "k", "stride", "pad", "cin", "cout", "kp")

    def __init__(self, conv: nn.Conv2d, bn: nn.BatchNorm2d, dt, kp=None):
        with torch.no_grad():
            inv = torch.rsqrt(bn.running_var.float() + BN_EPS) * bn.weight.float()
            w = conv.weight.float() * inv.view(-1, 1, 1, 1)              # fold the eval BN scale
            w = w.permute(0, 2, 3, 1).reshape(w.shape[0], -1)           # OIHW -> O(kh kw I)
            self.kp = kp or w.shape[1]
            if self.kp > w.shape[1]:
                w = torch.cat([w, w.new_zeros(w.shape[0], self.kp - w.shape[1])], 1)
            self.w = w.to(TORCH_DT[dt]).contiguous()
            self.b = (bn.bias.float() - bn.running_mean.float() * inv).contiguous()
        self.k, self.stride, self.pad = conv.kernel_size[0], conv.stride[0], conv.padding[0]
        self.cin, self.cout = conv.in_channels, conv.out_channels


class ResNet50Trunk(nn.Sequential):
    """``nn.Sequential(*list(torchvision.models.resnet50().children())[:-1])`` on HIP (inference)."""

    accepts_uint8_frames = True

    def __init__(self, compute_dtype: str = "fp32", input_normalization="imagenet"):
        mods = [nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False), nn.BatchNorm2d(64), nn.ReLU(inplace=True),
                nn.MaxPool2d(kernel_size=3, stride=2, padding=1)]
        inplanes = 64
        for i, (planes, blocks) in enumerate(zip(PLANES, LAYERS)):
            mods.append(_make_layer(inplanes, planes, blocks, 1 if i == 0 else 2))
            inplanes = planes * EXPANSION
        mods.append(nn.AdaptiveAvgPool2d((1, 1)))
        super().__init__(*mods)
        _torchvision_init_(self)
        if compute_dtype not in DTYPES:
            raise ValueError("compute_dtype must be 'fp32' or 'bf16'")
        self.compute_dtype = compute_dtype
        self.input_normalization = input_normalization
        self._folded = None
        self._folded_key = None

    # -- eval-mode BatchNorm folded into packed weights, rebuilt when any parameter/buffer changes
    def _state_key(self, dt):
        ts = list(self.parameters()) + [b for b in self.buffers()]
        return (dt, tuple((t.data_ptr(), t._version) for t in ts))

    def _fold(self, dt):
        key = self._state_key(dt)
        if self._folded is not None and self._folded_key == key:
            return self._folded
        f = {"stem": _Conv(self[0], self[1], dt, kp=STEM_KP), "layers": []}
        for li in range(4):
            blocks = []
            for blk in self[4 + li]:
                d = None if blk.downsample is None else _Conv(blk.downsample[0], blk.downsample[1], dt)
                blocks.append((_Conv(blk.conv1, blk.bn1, dt), _Conv(blk.conv2, blk.bn2, dt),
                               _Conv(blk.conv3, blk.bn3, dt), d))
            f["layers"].append(blocks)
        self._folded, self._folded_key = f, key
        return f

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """(N, 3, H, W) frames (fp32, or uint8 normalised in the conv1 gather) -> (N, 2048) fp32."""
        if self.training:
            raise NotImplementedError("the ResNet-50 ensemble member runs inference only on the MI355X path "
                                      "(call .eval(); training is provided for efficientnet_b0)")
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            raise NotImplementedError("no backward for the ResNet-50 member: run it under torch.no_grad() or "
                                      "freeze its parameters")
        _lib.require_hip(x, "frames")
        if x.dim() != 4 or x.shape[1] != 3:
            raise ValueError(f"expected (N, 3, H, W) frames, got {tuple(x.shape)}")
        if x.dtype not in (torch.float32, torch.uint8):
            x = x.float()
        dt = DTYPES[self.compute_dtype]
        with torch.no_grad():
            return _forward(self._fold(dt), x, dt, self.input_normalization)


def _norm6(spec) -> ctypes.Array:
    from .backbone import NORMALIZATIONS

    mean, std = NORMALIZATIONS[spec] if isinstance(spec, str) else spec
    return (ctypes.c_float * 6)(*[float(v) for v in mean], *[float(v) for v in std])


def _forward(f, x, dt, norm):
    lib = _lib.load()
    dev = x.device
    st = _lib.stream_of(dev)
    tdt = TORCH_DT[dt]
    N, _, H, W = x.shape

    def gemm(a, conv, m, res=None, relu=True):
        out = torch.empty(m, conv.cout, dtype=tdt, device=dev)
        _lib.check(lib.dfd_rn_gemm(st, dt, a.data_ptr(), conv.w.data_ptr(), out.data_ptr(), _lib.ptr(res),
                                   conv.b.data_ptr(), 1 if relu else 0, m, conv.cout, conv.kp))
        return out

    def conv(h, hw, c, res=None, relu=True):
        """one folded conv (+ identity) (+ ReLU): the implicit-GEMM MFMA kernel (k_rnconv.hip)"""
        (hh, ww) = hw
        ho = (hh + 2 * c.pad - c.k) // c.stride + 1
        wo = (ww + 2 * c.pad - c.k) // c.stride + 1
        out = torch.empty(N * ho * wo, c.cout, dtype=tdt, device=dev)
        _lib.check(lib.dfd_rn_conv(st, dt, h.data_ptr(), N, hh, ww, c.cin, c.k, c.k, c.stride, c.pad, c.w.data_ptr(),
                                   c.b.data_ptr(), _lib.ptr(res), 1 if relu else 0, c.cout, out.data_ptr()))
        return out, (ho, wo)

    # conv1 7x7/2 + bn1 + relu (frames gathered straight from the caller's tensor)
    stem = f["stem"]
    ho, wo = (H + 6 - 7) // 2 + 1, (W + 6 - 7) // 2 + 1
    a = torch.empty(N * ho * wo, STEM_KP, dtype=tdt, device=dev)
    fmt = 1 if x.dtype == torch.uint8 else 0
    _lib.check(lib.dfd_rn_stem_im2col(st, dt, x.data_ptr(), fmt, (ctypes.c_int64 * 4)(*x.stride()), _norm6(norm), N,
                                      H, W, a.data_ptr()))
    h = gemm(a, stem, N * ho * wo)
    # maxpool 3x3/2
    hp, wp = (ho + 2 - 3) // 2 + 1, (wo + 2 - 3) // 2 + 1
    p = torch.empty(N * hp * wp, 64, dtype=tdt, device=dev)
    _lib.check(lib.dfd_rn_maxpool(st, dt, h.data_ptr(), N, ho, wo, 64, p.data_ptr()))
    h, hw = p, (hp, wp)
    for blocks in f["layers"]:
        for c1, c2, c3, ds in blocks:
            identity = h if ds is None else conv(h, hw, ds, relu=False)[0]
            o, hw1 = conv(h, hw, c1)
            o, hw2 = conv(o, hw1, c2)
            h, hw = conv(o, hw2, c3, res=identity, relu=True)[0], hw2
    feats = torch.empty(N, FEATURE_DIM, dtype=torch.float32, device=dev)
    _lib.check(lib.dfd_rn_avgpool(st, dt, h.data_ptr(), N, hw[0] * hw[1], FEATURE_DIM, feats.data_ptr()))
    return feats


def resnet_state_names(trunk: nn.Module) -> List[str]:
    return [n for n, _ in trunk.state_dict().items()]
