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

TRAINING (``.train()``: ``EnsembleTrainer.train_epoch`` trains every member of the ensemble,
``src/ensemble_trainer.py:158-229``) runs in fp32 with torchvision's train-mode semantics -- batch
statistics (biased variance) normalise, the running buffers update with momentum 0.1 and the
unbiased variance, ``num_batches_tracked`` counts -- as one autograd node over the trunk
(``_RnTrainFn``): every convolution's forward, data gradient (stride 1 and 2) and weight gradient
are exact-fp32 implicit-GEMM MFMA kernels (``csrc/k_conv.hip``), the BatchNorm backward is the B0
path's reduce / finalize / apply (``csrc/k_bn.hip``), the ReLU / residual / pooling pieces are
``csrc/k_rntrain.hip`` and ``k_conv.hip`` kernels.  With ``compute_dtype='bf16'`` the member trains in
bf16 (round 6): conv1 + bn1 + relu + maxpool stay on those fp32 kernels, every bottleneck convolution
(forward with the BN-stat partials, data gradient at stride 1 and 2, weight gradient) runs on bf16 MFMA
over bf16 NHWC activations (``csrc/k_rn16.hip``: the EfficientNet-B0 1x1 GEMM tile loops reading an
implicit-GEMM gather), fp32 master weights packed to bf16 once per step, BatchNorm statistics and
coefficients in fp32 / fp64, the same train-mode semantics.
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

    def forward(self, x: torch.Tensor, grad_sink=None) -> torch.Tensor:
        """(N, 3, H, W) frames (fp32, or uint8 normalised in the conv1 gather) -> (N, 2048) fp32.
        grad_sink (training inside a FlatModule owner, e.g. the detector): the parameter gradients are
        written into its flat buffer."""
        _lib.require_hip(x, "frames")
        if x.dim() != 4 or x.shape[1] != 3:
            raise ValueError(f"expected (N, 3, H, W) frames, got {tuple(x.shape)}")
        grads = torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())
        if self.training:
            if x.dtype == torch.uint8:  # the serving feed's uint8 crops: normalise like the conv1 gather
                from .backbone import NORMALIZATIONS

                spec = self.input_normalization
                mean, std = NORMALIZATIONS[spec] if isinstance(spec, str) else spec
                x = (x.float() / 255.0 - torch.tensor(mean, device=x.device).view(1, 3, 1, 1)) / \
                    torch.tensor(std, device=x.device).view(1, 3, 1, 1)
            x = x.float()
            params = self.train_parameters()
            if grads:
                return _RnTrainFn.apply(x, self, grad_sink, *params)
            with torch.no_grad():
                return _train_forward(self, x, save=False)[0]
        if grads:
            raise NotImplementedError("no eval-mode backward for the ResNet-50 member (eval BatchNorm is folded "
                                      "into the inference kernels): train it in .train() mode or freeze it")
        if x.dtype not in (torch.float32, torch.uint8):
            x = x.float()
        dt = DTYPES[self.compute_dtype]
        with torch.no_grad():
            return _forward(self._fold(dt), x, dt, self.input_normalization)

    def train_units(self):
        """(conv, bn) pairs in forward order: stem, then per bottleneck conv1, conv2, conv3 (+ downsample)."""
        units = [(self[0], self[1])]
        for li in range(4):
            for blk in self[4 + li]:
                units += [(blk.conv1, blk.bn1), (blk.conv2, blk.bn2), (blk.conv3, blk.bn3)]
                if blk.downsample is not None:
                    units.append((blk.downsample[0], blk.downsample[1]))
        return units

    def train_parameters(self):
        out = []
        for conv, bn in self.train_units():
            out += [conv.weight, bn.weight, bn.bias]
        return out


# ------------------------------------------------------------------ training (fp32)
class _Unit:
    """One conv + train-mode BN of the trunk: the forward's saved tensors for the backward."""

    __slots__ = ("conv", "bn", "x", "hw", "y", "ohw", "mean", "invstd", "scale", "shift", "wd")


def _nhwc_strides(t, hw, c):
    return (ctypes.c_int64 * 4)(hw[0] * hw[1] * c, hw[1] * c, c, 1)


def _conv_bn_fwd(lib, st, u, x, xs, n, hw, save):
    """y = conv(x) (no bias), the BN batch statistics (running buffers updated) -> unit with scale/shift."""
    conv, bn = u.conv, u.bn
    k, s, p, cin, cout = conv.kernel_size[0], conv.stride[0], conv.padding[0], conv.in_channels, conv.out_channels
    ho, wo = (hw[0] + 2 * p - k) // s + 1, (hw[1] + 2 * p - k) // s + 1
    dev = x.device
    rows = lib.dfd_rn_conv_stat_rows(n, ho, wo)
    stats = torch.empty(rows * 2 * cout, dtype=torch.float32, device=dev)
    wpack = torch.empty(conv.weight.numel(), dtype=torch.float32, device=dev)
    y = torch.empty(n * ho * wo, cout, dtype=torch.float32, device=dev)
    w = conv.weight.detach().float().contiguous()
    _lib.check(lib.dfd_rn_train_conv_fwd(st, x.data_ptr(), xs, n, hw[0], hw[1], cin, w.data_ptr(), cout, k, k, s, p,
                                         wpack.data_ptr(), y.data_ptr(), stats.data_ptr()))
    vecs = torch.empty(4, cout, dtype=torch.float32, device=dev)
    with torch.no_grad():
        bn.num_batches_tracked.add_(1)
    # torch's momentum=None: the cumulative moving average, factor 1 / num_batches_tracked
    mom = float(bn.momentum) if bn.momentum is not None else 1.0 / float(bn.num_batches_tracked)
    _lib.check(lib.dfd_rn_bn_train_finalize(st, stats.data_ptr(), rows, n * ho * wo, cout, bn.weight.data_ptr(),
                                            bn.bias.data_ptr(), bn.running_mean.data_ptr(),
                                            bn.running_var.data_ptr(), mom, float(bn.eps),
                                            vecs[0].data_ptr(), vecs[1].data_ptr(), vecs[2].data_ptr(),
                                            vecs[3].data_ptr()))
    if save:
        u.x, u.hw, u.y, u.ohw = x, hw, y, (ho, wo)
        u.mean, u.invstd, u.scale, u.shift = vecs[0], vecs[1], vecs[2], vecs[3]
    return y, (ho, wo), vecs


def _bn_act(lib, st, y, vecs, bn, res, relu):
    """relu?((y - mean) * scale + beta (+ res)): torch's centred order of operations"""
    out = torch.empty_like(y)
    _lib.check(lib.dfd_rn_bn_act(st, y.data_ptr(), vecs[0].data_ptr(), vecs[2].data_ptr(), bn.bias.data_ptr(),
                                 _lib.ptr(res), 1 if relu else 0, y.shape[0], y.shape[1], out.data_ptr()))
    return out


def _bn_momentum(bn):
    with torch.no_grad():
        bn.num_batches_tracked.add_(1)
    # torch's momentum=None: the cumulative moving average, factor 1 / num_batches_tracked
    return float(bn.momentum) if bn.momentum is not None else 1.0 / float(bn.num_batches_tracked)


def _pack16(trunk, lib, st, dev, save):
    """Every bottleneck convolution's fp32 master weights -> bf16 wf (forward) and, for a backward, wd
    (data gradient) in ONE launch (dfd_rn16_pack_all) -> {id(conv): (wf, wd or None)} views of one buffer.
    The device table of weight pointers / shapes / offsets is built once per trunk and layout."""
    convs = []
    for li in range(4):
        for blk in trunk[4 + li]:
            convs += [blk.conv1, blk.conv2, blk.conv3] + ([blk.downsample[0]] if blk.downsample is not None else [])
    key = (bool(save), str(dev), tuple(c.weight.data_ptr() for c in convs))
    cache = getattr(trunk, "_rn16_pack", None)
    if cache is None or cache[0] != key:
        rows, off, spans = [], 0, []
        for c in convs:
            if c.weight.dtype != torch.float32 or not c.weight.is_contiguous():
                raise RuntimeError("bf16 ResNet training: conv weights must be contiguous fp32 masters")
            ne = c.weight.numel()
            kk = c.kernel_size[0] * c.kernel_size[1]
            od = off + ne if save else -1
            rows.append([c.weight.data_ptr(), c.out_channels, c.in_channels, kk, off, od])
            spans.append((off, od, ne))
            off += 2 * ne if save else ne
        table = torch.tensor(rows, dtype=torch.int64, device=dev)
        cache = (key, table, spans, off, max(sp[2] for sp in spans))
        trunk._rn16_pack = cache
    _, table, spans, total, mx = cache
    out = torch.empty(total, dtype=torch.bfloat16, device=dev)
    _lib.check(lib.dfd_rn16_pack_all(st, table.data_ptr(), len(convs), mx, out.data_ptr()))
    return {id(c): (out[o:o + ne], out[od:od + ne] if od >= 0 else None) for c, (o, od, ne) in zip(convs, spans)}


def _conv_bn_fwd16(lib, st, u, x, n, hw, save, packs):
    """bf16: y = conv(x) on the packed bf16 weights, the BN batch statistics (running buffers updated)."""
    conv, bn = u.conv, u.bn
    k, s, p, cin, cout = conv.kernel_size[0], conv.stride[0], conv.padding[0], conv.in_channels, conv.out_channels
    ho, wo = (hw[0] + 2 * p - k) // s + 1, (hw[1] + 2 * p - k) // s + 1
    dev = x.device
    wf, wd = packs[id(conv)]
    y = torch.empty(n * ho * wo, cout, dtype=torch.bfloat16, device=dev)
    stats = torch.empty(2048 * cout, dtype=torch.float32, device=dev)
    rows = ctypes.c_int(0)
    _lib.check(lib.dfd_rn16_conv_fwd(st, x.data_ptr(), n, hw[0], hw[1], cin, wf.data_ptr(), cout, k, s, p, y.data_ptr(),
                                     stats.data_ptr(), ctypes.byref(rows)))
    vecs = torch.empty(4, cout, dtype=torch.float32, device=dev)
    mom = _bn_momentum(bn)
    _lib.check(lib.dfd_rn16_bn_finalize(st, stats.data_ptr(), rows.value, n * ho * wo, cout, bn.weight.data_ptr(),
                                        bn.bias.data_ptr(), bn.running_mean.data_ptr(), bn.running_var.data_ptr(), mom,
                                        float(bn.eps), vecs[0].data_ptr(), vecs[1].data_ptr(), vecs[2].data_ptr(),
                                        vecs[3].data_ptr()))
    if save:
        u.x, u.hw, u.y, u.ohw, u.wd = x, hw, y, (ho, wo), wd
        u.mean, u.invstd, u.scale, u.shift = vecs[0], vecs[1], vecs[2], vecs[3]
    return y, (ho, wo), vecs


def _bn_act16(lib, st, y, vecs, bn, res, relu):
    out = torch.empty_like(y)
    _lib.check(lib.dfd_rn16_bn_act(st, y.data_ptr(), vecs[0].data_ptr(), vecs[2].data_ptr(), bn.bias.data_ptr(),
                                   _lib.ptr(res), 1 if relu else 0, y.shape[0], y.shape[1], out.data_ptr()))
    return out


def _train_forward(trunk, x, save):
    """Train-mode forward of the trunk -> (features (N, 2048), saved state for the backward)."""
    lib = _lib.load()
    dev = x.device
    st = _lib.stream_of(dev)
    n, _, H, W = x.shape
    units, blocks = [], []
    b16 = trunk.compute_dtype == "bf16"

    def unit(conv, bn):
        u = _Unit()
        u.conv, u.bn = conv, bn
        units.append(u)
        return u

    # conv1 7x7/2 reads the (N,3,H,W) frames through their strides; bn1 + relu + maxpool fused
    us = unit(trunk[0], trunk[1])
    xs = (ctypes.c_int64 * 4)(x.stride(0), x.stride(2), x.stride(3), x.stride(1))
    y0, hw0, v0 = _conv_bn_fwd(lib, st, us, x, xs, n, (H, W), save)
    hp, wp = (hw0[0] + 2 - 3) // 2 + 1, (hw0[1] + 2 - 3) // 2 + 1
    h = torch.empty(n * hp * wp, 64, dtype=torch.float32, device=dev)
    arg = torch.empty(n * hp * wp * 64, dtype=torch.uint8, device=dev)
    _lib.check(lib.dfd_rn_pool_train_fwd(st, y0.data_ptr(), v0[0].data_ptr(), v0[2].data_ptr(),
                                         trunk[1].bias.data_ptr(), n, hw0[0], hw0[1], 64,
                                         h.data_ptr(), arg.data_ptr()))
    hw = (hp, wp)
    if b16:  # the bottlenecks in bf16 (k_rn16.hip); the stem above stays fp32
        h16 = torch.empty(h.shape, dtype=torch.bfloat16, device=dev)
        _lib.check(lib.dfd_rn16_cast(st, h.data_ptr(), 1, h.numel(), h16.data_ptr()))
        h = h16
        packs = _pack16(trunk, lib, st, dev, save)
        for li in range(4):
            for blk in trunk[4 + li]:
                b = {"in": h, "hw": hw}
                u1, u2, u3 = unit(blk.conv1, blk.bn1), unit(blk.conv2, blk.bn2), unit(blk.conv3, blk.bn3)
                y1, hw1, v1 = _conv_bn_fwd16(lib, st, u1, h, n, hw, save, packs)
                a1 = _bn_act16(lib, st, y1, v1, blk.bn1, None, True)
                y2, hw2, v2 = _conv_bn_fwd16(lib, st, u2, a1, n, hw1, save, packs)
                a2 = _bn_act16(lib, st, y2, v2, blk.bn2, None, True)
                y3, _, v3 = _conv_bn_fwd16(lib, st, u3, a2, n, hw2, save, packs)
                if blk.downsample is not None:
                    ud = unit(blk.downsample[0], blk.downsample[1])
                    yd, _, vd = _conv_bn_fwd16(lib, st, ud, h, n, hw, save, packs)
                    idn = _bn_act16(lib, st, yd, vd, blk.downsample[1], None, False)
                    b["ds"] = ud
                else:
                    idn = h
                h = _bn_act16(lib, st, y3, v3, blk.bn3, idn, True)
                hw = hw2
                b.update(u=(u1, u2, u3), a1=a1, a2=a2, out=h)
                blocks.append(b)
    for li in range(0 if not b16 else 4, 4):
        for blk in trunk[4 + li]:
            b = {"in": h, "hw": hw}
            u1, u2, u3 = unit(blk.conv1, blk.bn1), unit(blk.conv2, blk.bn2), unit(blk.conv3, blk.bn3)
            y1, hw1, v1 = _conv_bn_fwd(lib, st, u1, h, _nhwc_strides(h, hw, blk.conv1.in_channels), n, hw, save)
            a1 = _bn_act(lib, st, y1, v1, blk.bn1, None, True)
            y2, hw2, v2 = _conv_bn_fwd(lib, st, u2, a1, _nhwc_strides(a1, hw1, blk.conv2.in_channels), n, hw1, save)
            a2 = _bn_act(lib, st, y2, v2, blk.bn2, None, True)
            y3, _, v3 = _conv_bn_fwd(lib, st, u3, a2, _nhwc_strides(a2, hw2, blk.conv3.in_channels), n, hw2, save)
            if blk.downsample is not None:
                ud = unit(blk.downsample[0], blk.downsample[1])
                yd, _, vd = _conv_bn_fwd(lib, st, ud, h, _nhwc_strides(h, hw, blk.conv1.in_channels), n, hw, save)
                idn = _bn_act(lib, st, yd, vd, blk.downsample[1], None, False)
                b["ds"] = ud
            else:
                idn = h
            h = _bn_act(lib, st, y3, v3, blk.bn3, idn, True)
            hw = hw2
            b.update(u=(u1, u2, u3), a1=a1, a2=a2, out=h)
            blocks.append(b)
    feats = torch.empty(n, FEATURE_DIM, dtype=torch.float32, device=dev)
    _lib.check(lib.dfd_rn_avgpool(st, 1 if b16 else 0, h.data_ptr(), n, hw[0] * hw[1], FEATURE_DIM, feats.data_ptr()))
    saved = dict(units=units, blocks=blocks, stem_arg=arg, stem_pool_hw=(hp, wp), final_hw=hw, n=n) if save else None
    return feats, saved


def _gdst(grads, p):
    """the gradient destination of parameter p: its view of the owner's flat gradient buffer when the
    trunk runs inside a FlatModule (GradSink; autograd adopts the views, no gather / scatter in the
    optimizer), else a new fp32 tensor"""
    t = grads.get(id(p))
    if t is None:
        t = torch.empty(p.shape, dtype=torch.float32, device=p.device)
        grads[id(p)] = t
    return t


def _bn_bwd(lib, st, u, g, grads, relu_out=None):
    """train-mode BN backward of unit u from its output gradient g -> dy; dgamma / dbeta into grads.
    relu_out: the saved output of the ReLU after this BN; g is then that ReLU's INPUT gradient, masked
    inside the kernels (never materialised)"""
    C = u.y.shape[1]
    dev = g.device
    stats = torch.empty(2048 * 2 * C, dtype=torch.float32, device=dev)
    coef = torch.empty(3 * C, dtype=torch.float32, device=dev)
    dg, db = _gdst(grads, u.bn.weight), _gdst(grads, u.bn.bias)
    dy = torch.empty_like(u.y)
    if relu_out is not None:
        _lib.check(lib.dfd_rn_bn_train_bwd_relu(st, g.data_ptr(), relu_out.data_ptr(), u.y.data_ptr(), u.y.shape[0], C,
                                                u.mean.data_ptr(), u.invstd.data_ptr(), u.bn.weight.data_ptr(),
                                                dg.data_ptr(), db.data_ptr(), stats.data_ptr(), coef.data_ptr(),
                                                dy.data_ptr()))
        return dy
    _lib.check(lib.dfd_rn_bn_train_bwd(st, g.data_ptr(), u.y.data_ptr(), u.y.shape[0], C, u.mean.data_ptr(),
                                       u.invstd.data_ptr(), u.scale.data_ptr(), u.shift.data_ptr(),
                                       u.bn.weight.data_ptr(), dg.data_ptr(), db.data_ptr(), stats.data_ptr(),
                                       coef.data_ptr(), dy.data_ptr()))
    return dy


def _conv_bwd(lib, st, u, dy, n, grads, need_dx=True, res=None):
    """data gradient (if needed; + res, the block's other path, added in the kernel's epilogue) and
    weight gradient of unit u's convolution from dy = dL/dy."""
    conv = u.conv
    k, s, p, cin, cout = conv.kernel_size[0], conv.stride[0], conv.padding[0], conv.in_channels, conv.out_channels
    dev = dy.device
    w = conv.weight.detach().float().contiguous()
    nw = w.numel()
    dx = None
    if need_dx:
        wp = torch.empty(2 * nw, dtype=torch.float32, device=dev)
        dx = torch.empty(n * u.hw[0] * u.hw[1], cin, dtype=torch.float32, device=dev)
        if res is not None:
            _lib.check(lib.dfd_rn_conv_dgrad_res(st, dy.data_ptr(), n, u.hw[0], u.hw[1], cin, w.data_ptr(), cout, k, k,
                                                 s, p, wp.data_ptr(), wp[nw:].data_ptr(), res.data_ptr(),
                                                 dx.data_ptr()))
        else:
            _lib.check(lib.dfd_rn_conv_dgrad(st, dy.data_ptr(), n, u.hw[0], u.hw[1], cin, w.data_ptr(), cout, k, k, s,
                                             p, wp.data_ptr(), wp[nw:].data_ptr(), dx.data_ptr()))
    slab = torch.empty(lib.dfd_rn_conv_wgrad_slab_floats(n, u.hw[0], u.hw[1], cin, cout, k, k, s, p),
                       dtype=torch.float32, device=dev)
    dw = _gdst(grads, conv.weight)
    x = u.x
    if x.dim() == 4:  # the stem reads the frames through their strides
        xs = (ctypes.c_int64 * 4)(x.stride(0), x.stride(2), x.stride(3), x.stride(1))
    else:
        xs = _nhwc_strides(x, u.hw, cin)
    _lib.check(lib.dfd_rn_conv_wgrad(st, x.data_ptr(), xs, n, u.hw[0], u.hw[1], cin, dy.data_ptr(), cout, k, k, s, p,
                                     slab.data_ptr(), slab.numel(), dw.data_ptr()))
    return dx


def _bn_bwd16(lib, st, u, g, grads, relu_out=None):
    """relu_out: the saved output of the ReLU after this BN; g is then its INPUT gradient, masked inline"""
    C = u.y.shape[1]
    dev = g.device
    stats = torch.empty(2048 * 2 * C, dtype=torch.float32, device=dev)
    coef = torch.empty(3 * C, dtype=torch.float32, device=dev)
    dg, db = _gdst(grads, u.bn.weight), _gdst(grads, u.bn.bias)
    dy = torch.empty_like(u.y)
    _lib.check(lib.dfd_rn16_bn_train_bwd(st, g.data_ptr(), _lib.ptr(relu_out), u.y.data_ptr(), u.y.shape[0], C,
                                         u.mean.data_ptr(),
                                         u.invstd.data_ptr(), u.scale.data_ptr(), u.shift.data_ptr(),
                                         u.bn.weight.data_ptr(), dg.data_ptr(), db.data_ptr(), stats.data_ptr(),
                                         coef.data_ptr(), dy.data_ptr()))
    return dy


def _conv_bwd16(lib, st, u, dy, n, grads, res=None):
    """bf16 data gradient (+ res: the other path's input gradient) and fp32 weight gradient of unit u."""
    conv = u.conv
    k, s, p, cin, cout = conv.kernel_size[0], conv.stride[0], conv.padding[0], conv.in_channels, conv.out_channels
    dev = dy.device
    dx = torch.empty(n * u.hw[0] * u.hw[1], cin, dtype=torch.bfloat16, device=dev)
    _lib.check(lib.dfd_rn16_conv_dgrad(st, dy.data_ptr(), n, u.hw[0], u.hw[1], cin, u.wd.data_ptr(), cout, k, s, p,
                                       _lib.ptr(res), dx.data_ptr()))
    slab = torch.empty(lib.dfd_rn16_conv_wgrad_slab_floats(n, u.hw[0], u.hw[1], cin, cout, k, s, p),
                       dtype=torch.float32, device=dev)
    dw = _gdst(grads, conv.weight)
    _lib.check(lib.dfd_rn16_conv_wgrad(st, u.x.data_ptr(), n, u.hw[0], u.hw[1], cin, dy.data_ptr(), cout, k, s, p,
                                       slab.data_ptr(), slab.numel(), dw.data_ptr()))
    return dx


def _relu_bwd16(lib, st, d, out):
    g = torch.empty_like(d)
    _lib.check(lib.dfd_rn16_relu_bwd(st, d.data_ptr(), out.data_ptr(), d.numel(), g.data_ptr()))
    return g


def _train_backward(trunk, saved, dfeat, grads=None):
    lib = _lib.load()
    dev = dfeat.device
    st = _lib.stream_of(dev)
    n = saved["n"]
    grads = {} if grads is None else grads
    blocks = saved["blocks"]
    hw = saved["final_hw"]
    if trunk.compute_dtype == "bf16":
        last = blocks[-1]["out"]
        g = torch.empty_like(last)
        _lib.check(lib.dfd_rn16_gap_bwd(st, dfeat.contiguous().data_ptr(), last.data_ptr(), n, hw[0] * hw[1],
                                        FEATURE_DIM, g.data_ptr()))
        for bi, b in enumerate(reversed(blocks)):
            u1, u2, u3 = b["u"]
            if bi > 0:  # the block's output ReLU (the last block's went with the pool)
                g = _relu_bwd16(lib, st, g, b["out"])
            dy3 = _bn_bwd16(lib, st, u3, g, grads)
            if "ds" in b:
                dyd = _bn_bwd16(lib, st, b["ds"], g, grads)
                other = _conv_bwd16(lib, st, b["ds"], dyd, n, grads)
            else:
                other = g
            # the ReLUs after bn2 / bn1 are folded into their BN backward (masked by the saved a2 / a1)
            dy2 = _bn_bwd16(lib, st, u2, _conv_bwd16(lib, st, u3, dy3, n, grads), grads, relu_out=b["a2"])
            dy1 = _bn_bwd16(lib, st, u1, _conv_bwd16(lib, st, u2, dy2, n, grads), grads, relu_out=b["a1"])
            g = _conv_bwd16(lib, st, u1, dy1, n, grads, res=other)
        g32 = torch.empty(g.shape, dtype=torch.float32, device=dev)
        _lib.check(lib.dfd_rn16_cast(st, g.data_ptr(), 0, g.numel(), g32.data_ptr()))
        return _stem_backward(lib, st, saved, g32, n, grads)
    # AdaptiveAvgPool2d + the last block's ReLU
    last = blocks[-1]["out"]
    g = torch.empty_like(last)
    _lib.check(lib.dfd_rn_gap_bwd(st, dfeat.contiguous().data_ptr(), last.data_ptr(), n, hw[0] * hw[1], FEATURE_DIM,
                                  g.data_ptr()))
    masked = True
    for b in reversed(blocks):
        u1, u2, u3 = b["u"]
        if not masked:  # the block's output ReLU
            gm = torch.empty_like(g)
            _lib.check(lib.dfd_rn_relu_bwd(st, g.data_ptr(), b["out"].data_ptr(), g.numel(), gm.data_ptr()))
            g = gm
        masked = False
        dy3 = _bn_bwd(lib, st, u3, g, grads)
        if "ds" in b:
            dyd = _bn_bwd(lib, st, b["ds"], g, grads)
            other = _conv_bwd(lib, st, b["ds"], dyd, n, grads)
        else:
            other = g  # the identity path
        da2 = _conv_bwd(lib, st, u3, dy3, n, grads)
        dy2 = _bn_bwd(lib, st, u2, da2, grads, relu_out=b["a2"])  # the ReLU after bn2 masked inside
        da1 = _conv_bwd(lib, st, u2, dy2, n, grads)
        dy1 = _bn_bwd(lib, st, u1, da1, grads, relu_out=b["a1"])
        g = _conv_bwd(lib, st, u1, dy1, n, grads, res=other)  # conv1's data gradient + the other path
    return _stem_backward(lib, st, saved, g, n, grads)


def _stem_backward(lib, st, saved, g, n, grads):
    """maxpool + stem relu/bn + conv1 weight gradient (fp32; no gradient to the frames)"""
    us = saved["units"][0]
    gs = torch.empty_like(us.y)
    _lib.check(lib.dfd_rn_pool_train_bwd(st, g.data_ptr(), saved["stem_arg"].data_ptr(), us.y.data_ptr(),
                                         us.mean.data_ptr(), us.scale.data_ptr(), us.bn.bias.data_ptr(), n,
                                         us.ohw[0], us.ohw[1], 64,
                                         gs.data_ptr()))
    dy0 = _bn_bwd(lib, st, us, gs, grads)
    _conv_bwd(lib, st, us, dy0, n, grads, need_dx=False)
    return grads


class _RnTrainFn(torch.autograd.Function):
    """The whole train-mode trunk as one autograd node: forward saves every unit's input, pre-BN
    output and batch statistics; backward returns the conv / BN parameter gradients (the frames get
    none: they are data)."""

    @staticmethod
    def forward(ctx, x, trunk, sink, *params):
        feats, saved = _train_forward(trunk, x, save=True)
        ctx.trunk, ctx.saved, ctx.nparams, ctx.sink = trunk, saved, len(params), sink
        return feats

    @staticmethod
    def backward(ctx, dfeat):
        if ctx.saved is None:
            raise RuntimeError("the ResNet-50 training node frees its saved activations after the first backward: "
                               "a second backward through it (retain_graph=True) is not supported")
        params = ctx.trunk.train_parameters()
        grads, span = {}, None
        if ctx.sink is not None:  # write straight into the owner's flat gradient buffer
            owner = ctx.sink.owner
            prefix = next(n for n, m in owner.named_modules() if m is ctx.trunk) + "."
            name_of = {id(p): prefix + n for n, p in ctx.trunk.named_parameters()}
            names = [name_of[id(p)] for p in params]
            for p, v in zip(params, ctx.sink.views(names)):
                grads[id(p)] = v
            offs = [owner._p_off[n] for n in names]
            span = (min(offs), max(o + p.numel() for o, p in zip(offs, params)))
        grads = _train_backward(ctx.trunk, ctx.saved, dfeat.float(), grads)
        ctx.saved = None
        if span is not None:
            ctx.sink.ready(*span)
        return (None, None, None) + tuple(grads.get(id(p)) for p in params)


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
    fmt = 1 if x.dtype == torch.uint8 else 0
    if dt == 1 and ho % 16 == 0 and wo % 16 == 0:
        # bf16: one implicit-GEMM launch (k_resnet.hip rn_stem_conv_kernel), no im2col rows in HBM
        h = torch.empty(N * ho * wo, stem.cout, dtype=tdt, device=dev)
        _lib.check(lib.dfd_rn_stem_conv(st, dt, x.data_ptr(), fmt, (ctypes.c_int64 * 4)(*x.stride()), _norm6(norm),
                                        N, H, W, stem.w.data_ptr(), stem.b.data_ptr(), h.data_ptr()))
    else:
        a = torch.empty(N * ho * wo, STEM_KP, dtype=tdt, device=dev)
        _lib.check(lib.dfd_rn_stem_im2col(st, dt, x.data_ptr(), fmt, (ctypes.c_int64 * 4)(*x.stride()), _norm6(norm),
                                          N, H, W, a.data_ptr()))
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
