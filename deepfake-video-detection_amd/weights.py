"""Portable deterministic weight generator (counter hash -> float).

Trained weights are unavailable (the reference checkpoint
``checkpoints/pretrained_dfdc200_20260125/checkpoint_best_efficientnet_b0.pt`` is a
Git-LFS pointer), so parity fixtures and the benchmark use
synthetic weights.  They are generated from ``(seed, tensor name, element index)``
with a splitmix64 counter hash in numpy, so the values are identical on every
machine and independent of the torch RNG -- the GPU box rebuilds the full-size
weights of a fixture instead of shipping 17 MB files.
"""
from __future__ import annotations

import zlib

import numpy as np

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_GOLD = np.uint64(0x9E3779B97F4A7C15)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + _GOLD
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def hash_uniform(seed: int, name: str, n: int) -> np.ndarray:
    """``n`` float32 values uniform in [-1, 1), a pure function of (seed, name, index)."""
    key = (zlib.crc32(name.encode()) & 0xFFFFFFFF) | ((seed & 0xFFFFFFFF) << 32)
    with np.errstate(over="ignore"):
        base = _splitmix64(np.array([key], dtype=np.uint64))[0]
        idx = np.arange(n, dtype=np.uint64) * _GOLD + base
    bits = _splitmix64(idx) >> np.uint64(40)  # 24 random bits
    return (bits.astype(np.float64) * (2.0 / (1 << 24)) - 1.0).astype(np.float32)


def init_value(seed: int, name: str, shape) -> np.ndarray:
    """Deterministic initial value for a parameter/buffer called ``name`` of ``shape``.

    Scales follow the usual fan-based recipes so activations stay O(1):
    conv/linear weights ``U(-1,1)*sqrt(3)*sqrt(2/fan_in)`` (depthwise: fan_in=k*k),
    biases ``0.05*U``, BN gamma ``1+0.1U``, beta ``0.1U``, running mean ``0.1U``,
    running var ``1+0.25|U|``.
    """
    shape = tuple(int(s) for s in shape)
    n = int(np.prod(shape)) if shape else 1
    u = hash_uniform(seed, name, n)
    leaf = name.rsplit(".", 1)[-1]
    if leaf == "num_batches_tracked":
        return np.zeros(shape, dtype=np.int64)
    if leaf == "running_mean":
        v = 0.1 * u
    elif leaf == "running_var":
        v = 1.0 + 0.25 * np.abs(u)
    elif leaf == "bias":
        v = 0.05 * u
    elif leaf == "weight" and len(shape) == 1:  # BN gamma
        v = 1.0 + 0.1 * u
    elif leaf == "weight":
        fan_in = int(np.prod(shape[1:])) if len(shape) > 1 else shape[0]
        v = u * np.sqrt(3.0) * np.sqrt(2.0 / max(1, fan_in))
    else:
        v = 0.1 * u
    return v.astype(np.float32).reshape(shape)


def deterministic_init_(module, seed: int = 0, prefix: str = "") -> None:
    """Overwrite every parameter and floating buffer of ``module`` in place (by state_dict name)."""
    import torch

    with torch.no_grad():
        for name, t in module.state_dict(keep_vars=True).items():
            full = prefix + name
            v = init_value(seed, full, t.shape)
            src = torch.from_numpy(v)
            if t.dtype == torch.int64:
                t.zero_()
            else:
                t.copy_(src.to(dtype=t.dtype))
