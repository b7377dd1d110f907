"""Plain PyTorch fp32 (CPU) restatement of timm ``efficientnet_b0`` -- ORACLE.

Test infrastructure only (see ``oracle/__init__.py``).

The reference builds its frame trunk with ``timm.create_model('efficientnet_b0')``
(``src/pretrained_detector.py:43``) and keeps ``children()[:-1]``
(``:46``): ``conv_stem, bn1, blocks, conv_head, bn2, global_pool``.  timm is
not vendored and not installed, so this module restates timm's published
architecture definition for ``efficientnet_b0``::

    ds_r1_k3_s1_e1_c16_se0.25
    ir_r2_k3_s2_e6_c24_se0.25
    ir_r2_k5_s2_e6_c40_se0.25
    ir_r3_k3_s2_e6_c80_se0.25
    ir_r3_k5_s1_e6_c112_se0.25
    ir_r4_k5_s2_e6_c192_se0.25
    ir_r1_k3_s1_e6_c320_se0.25

with timm's conventions: symmetric padding
``((s-1)+(k-1))//2``; BatchNorm eps 1e-5 / momentum 0.1 followed by SiLU
("BatchNormAct2d"); SE reduce width ``round(0.25 * block_in_chs)`` with SiLU and
a sigmoid gate, SE 1x1 convs with bias, every other conv bias-free; residual
when ``stride == 1 and in_chs == out_chs``; no drop-path.  Module attribute names
follow timm so ``state_dict`` keys match the keys the reference's checkpoint
loader expects (``app.py:1565`` heuristics ``conv_stem|.blocks.|conv_dw|se.conv``).

Parameter count (checked in tests): 4,007,548 trunk parameters.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

# (block_type, repeats, kernel, stride, expansion, out_chs) -- timm arch_def for B0
B0_ARCH = [
    ("ds", 1, 3, 1, 1, 16),
    ("ir", 2, 3, 2, 6, 24),
    ("ir", 2, 5, 2, 6, 40),
    ("ir", 3, 3, 2, 6, 80),
    ("ir", 3, 5, 1, 6, 112),
    ("ir", 4, 5, 2, 6, 192),
    ("ir", 1, 3, 1, 6, 320),
]
STEM_CHS = 32
HEAD_CHS = 1280


def _pad(k: int, s: int) -> int:
    return ((s - 1) + (k - 1)) // 2


class BatchNormAct2d(nn.BatchNorm2d):
    """timm ``BatchNormAct2d``: BatchNorm2d (eps 1e-5, momentum 0.1) + optional SiLU."""

    def __init__(self, c: int, act: bool = True):
        super().__init__(c, eps=1e-5, momentum=0.1)
        self.apply_act = act

    def forward(self, x):
        x = super().forward(x)
        return F.silu(x) if self.apply_act else x


class SqueezeExcite(nn.Module):
    """timm ``SqueezeExcite``: x * sigmoid(W_e SiLU(W_r mean_hw(x) + b_r) + b_e)."""

    def __init__(self, chs: int, rd: int):
        super().__init__()
        self.conv_reduce = nn.Conv2d(chs, rd, 1, bias=True)
        self.conv_expand = nn.Conv2d(rd, chs, 1, bias=True)

    def forward(self, x):
        s = x.mean((2, 3), keepdim=True)
        s = F.silu(self.conv_reduce(s))
        return x * torch.sigmoid(self.conv_expand(s))


class DepthwiseSeparableConv(nn.Module):
    """timm ``DepthwiseSeparableConv`` (stage 0): dw -> BN/SiLU -> SE -> pw -> BN."""

    def __init__(self, cin: int, cout: int, k: int, s: int):
        super().__init__()
        self.conv_dw = nn.Conv2d(cin, cin, k, s, _pad(k, s), groups=cin, bias=False)
        self.bn1 = BatchNormAct2d(cin, act=True)
        self.se = SqueezeExcite(cin, round(cin * 0.25))
        self.conv_pw = nn.Conv2d(cin, cout, 1, bias=False)
        self.bn2 = BatchNormAct2d(cout, act=False)
        self.has_skip = s == 1 and cin == cout

    def forward(self, x):
        sc = x
        x = self.bn1(self.conv_dw(x))
        x = self.se(x)
        x = self.bn2(self.conv_pw(x))
        return x + sc if self.has_skip else x


class InvertedResidual(nn.Module):
    """timm ``InvertedResidual``: pw -> BN/SiLU -> dw -> BN/SiLU -> SE -> pwl -> BN (+skip)."""

    def __init__(self, cin: int, cout: int, k: int, s: int, e: int):
        super().__init__()
        mid = cin * e
        self.conv_pw = nn.Conv2d(cin, mid, 1, bias=False)
        self.bn1 = BatchNormAct2d(mid, act=True)
        self.conv_dw = nn.Conv2d(mid, mid, k, s, _pad(k, s), groups=mid, bias=False)
        self.bn2 = BatchNormAct2d(mid, act=True)
        # se_ratio 0.25 is relative to the block input width (timm se_from_exp=False)
        self.se = SqueezeExcite(mid, round(cin * 0.25))
        self.conv_pwl = nn.Conv2d(mid, cout, 1, bias=False)
        self.bn3 = BatchNormAct2d(cout, act=False)
        self.has_skip = s == 1 and cin == cout

    def forward(self, x):
        sc = x
        x = self.bn1(self.conv_pw(x))
        x = self.bn2(self.conv_dw(x))
        x = self.se(x)
        x = self.bn3(self.conv_pwl(x))
        return x + sc if self.has_skip else x


class SelectAdaptivePool2d(nn.Module):
    """timm global pool ('avg', flatten=True)."""

    def forward(self, x):
        return x.mean((2, 3))


def block_specs():
    """Yield (stage, idx, type, cin, cout, k, s, e) for the 16 MBConv blocks."""
    cin = STEM_CHS
    for si, (bt, r, k, s, e, cout) in enumerate(B0_ARCH):
        for bi in range(r):
            stride = s if bi == 0 else 1
            yield si, bi, bt, cin, cout, k, stride, e
            cin = cout


class EfficientNetB0(nn.Module):
    """timm-topology EfficientNet-B0 with a 1000-way classifier (dropped by the detector)."""

    def __init__(self, num_classes: int = 1000):
        super().__init__()
        self.conv_stem = nn.Conv2d(3, STEM_CHS, 3, 2, _pad(3, 2), bias=False)
        self.bn1 = BatchNormAct2d(STEM_CHS, act=True)
        stages = []
        cur = []
        last_stage = 0
        for si, bi, bt, cin, cout, k, s, e in block_specs():
            if si != last_stage:
                stages.append(nn.Sequential(*cur))
                cur, last_stage = [], si
            if bt == "ds":
                cur.append(DepthwiseSeparableConv(cin, cout, k, s))
            else:
                cur.append(InvertedResidual(cin, cout, k, s, e))
        stages.append(nn.Sequential(*cur))
        self.blocks = nn.Sequential(*stages)
        self.conv_head = nn.Conv2d(320, HEAD_CHS, 1, bias=False)
        self.bn2 = BatchNormAct2d(HEAD_CHS, act=True)
        self.global_pool = SelectAdaptivePool2d()
        self.classifier = nn.Linear(HEAD_CHS, num_classes)

    def forward(self, x):
        x = self.bn1(self.conv_stem(x))
        x = self.blocks(x)
        x = self.bn2(self.conv_head(x))
        x = self.global_pool(x)
        return self.classifier(x)


def create_model(name: str = "efficientnet_b0", pretrained: bool = False, **_kw):
    """Stand-in for ``timm.create_model`` used only by the golden generator's timm stub."""
    if name != "efficientnet_b0":
        raise ValueError(f"oracle only restates efficientnet_b0, got {name}")
    if pretrained:
        raise RuntimeError("pretrained weights are unavailable offline")
    return EfficientNetB0()


def trunk(model: EfficientNetB0) -> nn.Sequential:
    """The reference's ``nn.Sequential(*list(backbone.children())[:-1])`` (pretrained_detector.py:46)."""
    return nn.Sequential(*list(model.children())[:-1])
