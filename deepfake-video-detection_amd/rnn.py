"""Drop-in ``LogicRNNLSTM`` / ``LogicCell`` / ``create_model`` on MI355X (src/RNNModel.py).

Same constructor arguments, submodule names and ``state_dict`` keys as the reference
(``logic_cells.{i}.{and,or,not,forget,input,cell,output}_gate.{weight,bias}``,
``attention.{0,2}.*``, ``classifier.{0,3}.*``), same ``forward(x, lengths=None)`` ->
``sigmoid`` output of shape ``(B, 1)`` and ``predict``.  Reference quirks are kept
(SURVEY F8c/F8d): the batch is sorted by ``lengths`` and never un-sorted (``RNNModel.py:92-95``)
and all layers share one ``(h, c)`` per time step (``:103-115``).

The recurrence, attention pooling and classifier run in fp32 HIP kernels behind the C ABI
(``dfd_rnn_forward`` / ``dfd_rnn_backward``, ``csrc/k_rnn.hip``); parameters live in one flat
fp32 buffer so gradients land in one flat tensor.  Dropout uses the library's counter hash
(bit-for-bit different from torch's RNG stream, identical in distribution); parity runs use
``dropout=0`` or ``eval()`` as the reference goldens do.
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn as nn

from . import _lib
from .flat import FlatModule, GradSink


class LogicCell(nn.Module):
    """``LogicCell`` (src/RNNModel.py:5-41): parameters only; the math runs in ``csrc/k_rnn.hip``."""

    def __init__(self, input_size, hidden_size):
        super().__init__()
        self.hidden_size = hidden_size
        self.and_gate = nn.Linear(input_size + hidden_size, hidden_size)
        self.or_gate = nn.Linear(input_size + hidden_size, hidden_size)
        self.not_gate = nn.Linear(hidden_size, hidden_size)
        self.forget_gate = nn.Linear(input_size + hidden_size, hidden_size)
        self.input_gate = nn.Linear(input_size + hidden_size, hidden_size)
        self.cell_gate = nn.Linear(input_size + hidden_size, hidden_size)
        self.output_gate = nn.Linear(input_size + hidden_size, hidden_size)


class LogicRNNLSTM(FlatModule):
    def __init__(self, input_size=1024, hidden_size=512, num_layers=2, dropout=0.5):
        super().__init__()
        if not 1 <= num_layers <= 8:
            raise ValueError("num_layers must be in 1..8")
        self.input_size = input_size
        self.hidden_size = hidden_size
        self.num_layers = num_layers
        self.logic_cells = nn.ModuleList([LogicCell(input_size if i == 0 else hidden_size, hidden_size)
                                          for i in range(num_layers)])
        self.dropout = nn.Dropout(dropout)
        self.attention = nn.Sequential(nn.Linear(hidden_size, hidden_size), nn.Tanh(), nn.Linear(hidden_size, 1),
                                       nn.Softmax(dim=1))
        self.classifier = nn.Sequential(nn.Linear(hidden_size, hidden_size), nn.ReLU(), nn.Dropout(dropout),
                                        nn.Linear(hidden_size, 1))
        self._flatten()

    def _on_flatten(self) -> None:
        self._names = [n for n, _ in self._flat_params]

    def forward(self, x: torch.Tensor, lengths: torch.Tensor | None = None) -> torch.Tensor:
        self.ensure_flat()
        _lib.require_hip(x, "x")
        if x.dim() != 3 or x.shape[2] != self.input_size:
            raise ValueError(f"expected (B, T, {self.input_size}), got {tuple(x.shape)}")
        x = x.float().contiguous()
        B, T, _ = x.shape
        order = lens = None
        if lengths is not None:
            lengths = torch.as_tensor(lengths, device=x.device)
            lens, order = lengths.sort(0, descending=True)  # RNNModel.py:92-95 (no un-sort later)
            lens, order = lens.to(torch.int64).contiguous(), order.contiguous()
        p = float(self.dropout.p) if self.training else 0.0
        seed = int(torch.randint(0, 2**62, (1,)).item()) if p > 0 else 0
        params = [p_ for _, p_ in self._flat_params]
        need_grad = torch.is_grad_enabled() and any(q.requires_grad for q in params)
        if not need_grad:
            return _rnn_forward(self, x, order, lens, seed, p)[0]
        return _RnnFn.apply(x, order, lens, self, GradSink(self), seed, p, *params)

    def predict(self, x, lengths=None):
        with torch.no_grad():
            return (self.forward(x, lengths) >= 0.5).float()


def create_model(config=None):
    """``create_model`` (src/RNNModel.py:149-170)."""
    if config is None:
        config = {"input_size": 1024, "hidden_size": 512, "num_layers": 2, "dropout": 0.5}
    return LogicRNNLSTM(input_size=config.get("input_size", 1024), hidden_size=config.get("hidden_size", 512),
                        num_layers=config.get("num_layers", 2), dropout=config.get("dropout", 0.5))


def _ptrs(tensors) -> ctypes.Array:
    arr = (ctypes.c_void_p * len(tensors))()
    for i, t in enumerate(tensors):
        arr[i] = t.data_ptr()
    return arr


def _dims(m: LogicRNNLSTM, x):
    B, T, _ = x.shape
    return B, T, m.input_size, m.hidden_size, m.num_layers


def _rnn_forward(m: LogicRNNLSTM, x, order, lens, seed, p):
    lib = _lib.load()
    dev = x.device
    d = _dims(m, x)
    work = torch.empty(int(lib.dfd_rnn_work_floats(*d)), dtype=torch.float32, device=dev)
    y = torch.empty(d[0], 1, dtype=torch.float32, device=dev)
    params = [p_ for _, p_ in m._flat_params]
    _lib.check(lib.dfd_rnn_forward(_lib.stream_of(dev), *d, x.data_ptr(), _lib.ptr(order), _lib.ptr(lens),
                                   _ptrs(params), work.data_ptr(), y.data_ptr(), seed, p))
    return y, work


class _RnnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, order, lens, m, sink, seed, p, *params):
        y, work = _rnn_forward(m, x, order, lens, seed, p)
        ctx.m, ctx.sink, ctx.seed, ctx.p, ctx.work = m, sink, seed, p, work
        ctx.x, ctx.order, ctx.lens = x, order, lens
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        m = ctx.m
        lib = _lib.load()
        x = ctx.x
        dev = x.device
        d = _dims(m, x)
        dy = dy.contiguous().float()
        scratch = torch.empty(int(lib.dfd_rnn_scratch_floats(*d)), dtype=torch.float32, device=dev)
        gviews = ctx.sink.views(m._names)
        params = [p_ for _, p_ in m._flat_params]
        _lib.check(lib.dfd_rnn_backward(_lib.stream_of(dev), *d, x.data_ptr(), _lib.ptr(ctx.order),
                                        _lib.ptr(ctx.lens), _ptrs(params), ctx.work.data_ptr(), scratch.data_ptr(),
                                        dy.data_ptr(), _ptrs(gviews), ctx.seed, ctx.p))
        ctx.work = None
        return (None, None, None, None, None, None, None, *gviews)
