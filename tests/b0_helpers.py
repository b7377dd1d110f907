"""Shared helpers for the EfficientNet-B0 parity tests (oracle side + introspection)."""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from deepfake_amd import _lib
from deepfake_amd.weights import deterministic_init_, hash_uniform
from oracle import b0_cpu


def oracle_trunk(seed: int) -> torch.nn.Sequential:
    t = b0_cpu.trunk(b0_cpu.EfficientNetB0())
    deterministic_init_(t, seed=seed, prefix="backbone.")
    return t


def frames(seed, shape):
    """Same synthetic ImageNet-normalised frames as tests/golden/make_golden.py."""
    n = int(np.prod(shape))
    u = (hash_uniform(seed, "frames", n) + 1.0) * 0.5
    x = torch.from_numpy(u.reshape(shape))
    mean = torch.tensor([0.485, 0.456, 0.406]).view(1, 1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225]).view(1, 1, 3, 1, 1)
    return ((x - mean) / std).float()


def oracle_saved(trunk: torch.nn.Sequential, x: torch.Tensor):
    """Pre-BN conv outputs and block outputs of the oracle, in the order of dfd_b0_saved_tensor,
    as NHWC [rows][cols] float tensors."""
    outs = []
    hooks = []

    def grab(_m, _i, o):
        outs.append(o.detach().permute(0, 2, 3, 1).reshape(-1, o.shape[1]).clone())

    hooks.append(trunk[0].register_forward_hook(grab))
    for stage in trunk[2]:
        for blk in stage:
            if isinstance(blk, b0_cpu.DepthwiseSeparableConv):
                mods = [blk.conv_dw, blk.conv_pw]
            else:
                mods = [blk.conv_pw, blk.conv_dw, blk.conv_pwl]
            for m in mods:
                hooks.append(m.register_forward_hook(grab))
            hooks.append(blk.register_forward_hook(grab))
    hooks.append(trunk[3].register_forward_hook(grab))
    feats = trunk(x)
    for h in hooks:
        h.remove()
    return outs, feats


def hip_saved(runtime, plan, ws: torch.Tensor, dtype: int):
    lib = _lib.load()
    off, rows, cols = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    out = []
    i = 0
    tdt = torch.float32 if dtype == 0 else torch.bfloat16
    es = 4 if dtype == 0 else 2
    while lib.dfd_b0_saved_tensor(plan, i, ctypes.byref(off), ctypes.byref(rows), ctypes.byref(cols)) == 0:
        n = rows.value * cols.value
        t = ws[off.value:off.value + n * es].view(tdt).view(rows.value, cols.value).float().cpu()
        out.append(t)
        i += 1
    return out


def rel_err(a: torch.Tensor, b: torch.Tensor) -> float:
    a = a.double()
    b = b.double()
    return float((a - b).norm() / (b.norm() + 1e-30))
