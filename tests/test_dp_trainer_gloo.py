"""``DataParallelTrainer`` through its REAL constructor and hook path, two gloo ranks on CPU.

The model is a small ``FlatModule`` whose backward behaves like the HIP detector's: gradients are
written into one ``GradSink`` buffer and announced segment by segment in reverse flat order
(head first, then the trunk's stages from the last to the stem -- the B0 segment order of
``backbone._TrunkFn.backward``), before autograd adopts the sink views as ``p.grad``.  Checked:

* bucket launches follow the segments (adjacent ranges merged until ``bucket_elems``);
* after ``forward_backward`` + ``sync_grads`` every ``p.grad`` is the sink view and equals the
  MEAN over ranks of the single-process gradients of each rank's shard (loss
  pre-divided by the world size, SUM all-reduce);
* parameters are broadcast from rank 0 at construction;
* a stale ``.grad`` at backward (gradient accumulation) raises instead of silently diverging.

The criterion is injected (``TrainStep(criterion=...)``, like the reference's ``train_epoch``
receives it) because the default HIP cross entropy needs a GPU; the optimizer is not stepped.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

from deepfake_amd.flat import FlatModule, GradSink
from deepfake_amd.trainer import DataParallelTrainer

D, NC = 24, 2
# (lo, hi) flat ranges announced in this order: "head" (b), then "stages" of w from the last rows
SEGMENTS = [(D * NC, D * NC + NC), (D * NC // 2, D * NC), (D * NC // 4, D * NC // 2), (0, D * NC // 4)]


class _SegmentedLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, model, sink, w, b):
        ctx.save_for_backward(x, w)
        ctx.model, ctx.sink = model, sink
        return torch.tanh(x @ w) + b

    @staticmethod
    def backward(ctx, gout):
        x, w = ctx.saved_tensors
        g = ctx.sink.get()
        dz = gout * (1 - torch.tanh(x @ w) ** 2)
        gw = (x.t() @ dz).reshape(-1)
        gb = gout.sum(0)
        g[: D * NC].copy_(gw)
        g[D * NC:].copy_(gb)
        for lo, hi in SEGMENTS:
            ctx.sink.ready(lo, hi)
        gwv, gbv = ctx.sink.views(["w", "b"])
        return None, None, None, gwv, gbv


class MiniDetector(FlatModule):
    def __init__(self, seed):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.w = nn.Parameter(torch.randn(D, NC, generator=g) * 0.3)
        self.b = nn.Parameter(torch.randn(NC, generator=g) * 0.1)
        self._grad_ready_hooks = []
        self._flatten()

    def register_grad_ready_hook(self, fn):
        self._grad_ready_hooks.append(fn)
        return fn

    def forward(self, x):
        self.ensure_flat()
        sink = GradSink(self)
        return _SegmentedLinear.apply(x, self, sink, self.w, self.b), None


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard(rank):
    g = torch.Generator().manual_seed(100 + rank)
    return torch.randn(6, D, generator=g), torch.randint(0, NC, (6,), generator=g)


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = {}
        model = MiniDetector(seed=rank)  # different init per rank: the broadcast must align them
        tr = DataParallelTrainer(model, bucket_elems=D * NC // 2 + 1, criterion=nn.CrossEntropyLoss())
        launched = []
        orig = tr._launch
        tr._launch = lambda flat, lo, hi: (launched.append((lo, hi)), orig(flat, lo, hi))
        out["w0"] = model.w.detach().numpy().copy()  # numpy: tensors through a Queue need the sender alive
        x, y = _shard(rank)
        loss, _ = tr.forward_backward(x, y)
        tr.sync_grads()
        out["launched"] = launched
        out["adopted"] = bool(model.w.grad.data_ptr() == tr._flat.data_ptr()
                              and model.b.grad.data_ptr() == tr._flat[D * NC:].data_ptr())
        out["gw"], out["gb"] = model.w.grad.numpy().copy(), model.b.grad.numpy().copy()
        # stale .grad at backward -> refused
        model.w.grad = torch.zeros_like(model.w)
        try:
            o, _ = model(x)
            (nn.functional.cross_entropy(o, y) / world).backward()
            out["stale_raised"] = False
        except RuntimeError as e:
            out["stale_raised"] = "set_to_none" in str(e)
        tr._works.clear()
        tr._pending = None
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_dp_trainer_real_hook_path_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=150) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # reference: rank 0's weights, mean of the per-shard single-process gradients
    ref = MiniDetector(seed=0)
    gw = torch.zeros_like(ref.w)
    gb = torch.zeros_like(ref.b)
    for r in range(world):
        w = ref.w.detach().clone().requires_grad_(True)
        b = ref.b.detach().clone().requires_grad_(True)
        x, y = _shard(r)
        nn.functional.cross_entropy(torch.tanh(x @ w) + b, y).backward()
        gw += w.grad / world
        gb += b.grad / world
    for r in range(world):
        o = res[r]
        assert torch.equal(torch.from_numpy(o["w0"]), ref.w.detach())
        # head segment + first stage merge (adjacent) until >= bucket_elems, then the rest
        assert o["launched"] == [(SEGMENTS[1][0], SEGMENTS[0][1]), (0, SEGMENTS[1][0])], o["launched"]
        assert o["adopted"]
        torch.testing.assert_close(torch.from_numpy(o["gw"]), gw, rtol=1e-6, atol=1e-7)
        torch.testing.assert_close(torch.from_numpy(o["gb"]), gb, rtol=1e-6, atol=1e-7)
        assert o["stale_raised"]
