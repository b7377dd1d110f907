"""Drop-in ``CNNLSTMHybrid`` on MI355X (src/models.py:20-85).

Same constructor, submodules and ``state_dict`` keys as the reference (``cnn.{0,1,4,5,8,9,12,13}.*``,
``lstm.*_l{k}``, ``attention.{0,2}.*``, ``classifier.{0,3}.*``) and the same
``forward(x (B, T, 3, H, W)) -> logits (B, num_classes)``.  The frame CNN (implicit-GEMM convs on
fp32 MFMA, fused BN+ReLU+MaxPool / BN+ReLU+GAP), the LSTM stack, attention pooling and classifier
run in HIP behind ``dfd_cnnlstm_forward/backward`` (``csrc/cnnlstm.cpp``); parameters and BN
running statistics live in flat buffers (gradients land in one flat tensor).  Dropout uses the
library's counter hash (same distribution as torch's, different stream); parity runs use
``dropout=0`` / ``eval()`` like the reference goldens.
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn as nn

from . import _lib
from .flat import FlatModule, GradSink

_BN_IDX = (1, 5, 9, 13)


class CNNLSTMHybrid(FlatModule):
    def __init__(self, input_channels=3, hidden_size=256, num_layers=2, num_classes=2, dropout=0.3):
        super().__init__()
        if input_channels != 3:
            raise ValueError("the HIP frame CNN takes 3-channel frames")
        if hidden_size % 8 or not 1 <= num_layers <= 8:
            raise ValueError("hidden_size must be a multiple of 8 and num_layers in 1..8")
        self.hidden_size = hidden_size
        self.num_layers = num_layers
        self.num_classes = num_classes
        self.cnn = nn.Sequential(
            nn.Conv2d(input_channels, 64, kernel_size=7, stride=2, padding=3), nn.BatchNorm2d(64), nn.ReLU(),
            nn.MaxPool2d(kernel_size=3, stride=2, padding=1),
            nn.Conv2d(64, 128, kernel_size=5, stride=1, padding=2), nn.BatchNorm2d(128), nn.ReLU(),
            nn.MaxPool2d(kernel_size=3, stride=2, padding=1),
            nn.Conv2d(128, 256, kernel_size=3, stride=1, padding=1), nn.BatchNorm2d(256), nn.ReLU(),
            nn.MaxPool2d(kernel_size=3, stride=2, padding=1),
            nn.Conv2d(256, 512, kernel_size=3, stride=1, padding=1), nn.BatchNorm2d(512), nn.ReLU(),
            nn.AdaptiveAvgPool2d(1), nn.Flatten())
        self.cnn_out_features = 512
        self.lstm = nn.LSTM(input_size=512, hidden_size=hidden_size, num_layers=num_layers,
                            dropout=dropout if num_layers > 1 else 0, batch_first=True)
        self.attention = nn.Sequential(nn.Linear(hidden_size, hidden_size), nn.Tanh(), nn.Linear(hidden_size, 1))
        self.classifier = nn.Sequential(nn.Linear(hidden_size, 128), nn.ReLU(), nn.Dropout(dropout),
                                        nn.Linear(128, num_classes))
        self._flatten()

    def _on_flatten(self) -> None:
        self._names = [n for n, _ in self._flat_params]
        bufs = dict(self.named_buffers())  # after flattening: views into the flat BN buffer
        self._bn_run = [bufs[f"cnn.{i}.{k}"] for i in _BN_IDX for k in ("running_mean", "running_var")]

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        self.ensure_flat()
        _lib.require_hip(x, "x")
        if x.dim() != 5 or x.shape[2] != 3:
            raise ValueError(f"expected (B, T, 3, H, W), got {tuple(x.shape)}")
        B, T, C, H, W = x.shape
        frames = x.reshape(B * T, C, H, W).float()
        training = self.training
        if training:
            with torch.no_grad():
                for i in _BN_IDX:
                    self.cnn[i].num_batches_tracked.add_(1)
        p = float(self.classifier[2].p) if training else 0.0
        seed = int(torch.randint(0, 2**62, (1,)).item()) if p > 0 else 0
        params = [q for _, q in self._flat_params]
        need_grad = torch.is_grad_enabled() and any(q.requires_grad for q in params)
        dims = (B, T, H, W, self.hidden_size, self.num_layers, self.num_classes)
        if not need_grad:
            return _cl_forward(self, frames, dims, training, seed, p)[0]
        return _ClFn.apply(frames, self, GradSink(self), dims, training, seed, p, *params)


def _ptrs(tensors) -> ctypes.Array:
    arr = (ctypes.c_void_p * len(tensors))()
    for i, t in enumerate(tensors):
        arr[i] = t.data_ptr()
    return arr


def _cl_forward(m: CNNLSTMHybrid, frames, dims, training, seed, p):
    lib = _lib.load()
    dev = frames.device
    work = torch.empty(int(lib.dfd_cnnlstm_work_floats(*dims)), dtype=torch.float32, device=dev)
    logits = torch.empty(dims[0], dims[6], dtype=torch.float32, device=dev)
    xs = (ctypes.c_int64 * 4)(*frames.stride())
    momentum = m.cnn[1].momentum if m.cnn[1].momentum is not None else 0.1
    _lib.check(lib.dfd_cnnlstm_forward(_lib.stream_of(dev), *dims, frames.data_ptr(), xs,
                                       _ptrs([q for _, q in m._flat_params]), _ptrs(m._bn_run), work.data_ptr(),
                                       1 if training else 0, float(momentum), seed, p, logits.data_ptr()))
    return logits, work


class _ClFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, frames, m, sink, dims, training, seed, p, *params):
        logits, work = _cl_forward(m, frames, dims, training, seed, p)
        ctx.m, ctx.sink, ctx.dims, ctx.training, ctx.seed, ctx.p, ctx.work = m, sink, dims, training, seed, p, work
        ctx.frames = frames
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        m = ctx.m
        lib = _lib.load()
        frames = ctx.frames
        dev = frames.device
        dlogits = dlogits.contiguous().float()
        scratch = torch.empty(int(lib.dfd_cnnlstm_scratch_floats(*ctx.dims)), dtype=torch.float32, device=dev)
        gviews = ctx.sink.views(m._names)
        xs = (ctypes.c_int64 * 4)(*frames.stride())
        _lib.check(lib.dfd_cnnlstm_backward(_lib.stream_of(dev), *ctx.dims, frames.data_ptr(), xs,
                                            _ptrs([q for _, q in m._flat_params]), ctx.work.data_ptr(),
                                            scratch.data_ptr(), 1 if ctx.training else 0, ctx.seed, ctx.p,
                                            dlogits.data_ptr(), _ptrs(gviews)))
        ctx.work = None
        return (None, None, None, None, None, None, None, *gviews)
