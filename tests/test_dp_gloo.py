"""Data-parallel gradient exchange of ``DataParallelTrainer`` on CPU (gloo, world size 2).

The GPU path uses the same code over RCCL ("nccl" backend) with one process per GPU; here the
bucketing of the grad-ready segments (reverse flat order: head, conv_head, stage 6, ...) and
the async all-reduce + wait are exercised with two gloo ranks on 127.0.0.1.  Reference
semantics: the loss is pre-divided by the world size, so the summed gradient
is the mean of the per-shard gradients; BN statistics stay local; parameters are broadcast
from rank 0 at construction.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from deepfake_amd.trainer import DataParallelTrainer


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bare_trainer(bucket_elems):
    tr = DataParallelTrainer.__new__(DataParallelTrainer)
    tr.world_size = dist.get_world_size()
    tr.pg = None
    tr.bucket_elems = bucket_elems
    tr._works, tr._pending, tr._flat = [], None, None
    tr.model = torch.nn.Module()  # no parameters: the adoption check has nothing to inspect
    tr.comm_enabled, tr.bucket_log = True, []
    return tr


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = {}
        # --- bucketing + all-reduce of a flat gradient, segments arriving in reverse order ---
        tr = _bare_trainer(bucket_elems=30)
        launched = []
        orig = tr._launch
        tr._launch = lambda flat, lo, hi: (launched.append((lo, hi)), orig(flat, lo, hi))
        flat = torch.arange(100, dtype=torch.float32) * (rank + 1)
        for lo, hi in [(80, 100), (60, 80), (10, 60), (0, 10)]:
            tr._on_ready(flat, lo, hi)
        tr.sync_grads()
        out["launched"] = launched
        out["flat_ok"] = bool(torch.equal(flat, torch.arange(100, dtype=torch.float32) * sum(range(1, world + 1))))
        # --- non-adjacent segment flushes the pending bucket ---
        tr = _bare_trainer(bucket_elems=1000)
        launched2 = []
        orig2 = tr._launch
        tr._launch = lambda flat, lo, hi: (launched2.append((lo, hi)), orig2(flat, lo, hi))
        flat2 = torch.ones(50) * (rank + 1)
        tr._on_ready(flat2, 40, 50)
        tr._on_ready(flat2, 0, 20)  # gap [20, 40) -> flush (40, 50)
        tr.sync_grads()
        out["launched2"] = launched2
        out["flat2"] = flat2.tolist()
        # --- loss / world then SUM == mean of per-shard gradients ---
        torch.manual_seed(0)
        w = torch.nn.Parameter(torch.randn(4, 3))
        xs = [torch.randn(5, 3) for _ in range(world)]
        ((xs[rank] @ w.t()).pow(2).mean() / world).backward()
        dist.all_reduce(w.grad)
        ref = torch.zeros_like(w)
        for x in xs:
            w2 = w.detach().clone().requires_grad_(True)
            (x @ w2.t()).pow(2).mean().backward()
            ref += w2.grad / world
        out["mean_ok"] = bool(torch.allclose(w.grad, ref, rtol=1e-6, atol=1e-7))
        # --- parameter / BN-buffer broadcast from rank 0 at construction ---
        class _M:
            pass

        m = _M()
        m._flat_p = torch.full((7,), float(rank + 5))
        m._flat_b = torch.full((3,), float(rank + 9))
        tr = _bare_trainer(1)
        tr.model = m
        tr._broadcast_params()
        out["bcast"] = (m._flat_p.tolist(), m._flat_b.tolist())
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_dp_bucketed_allreduce_gloo_world2():
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
    for r in range(world):
        o = res[r]
        assert o["launched"] == [(60, 100), (10, 60), (0, 10)]
        assert o["flat_ok"]
        assert o["launched2"] == [(40, 50), (0, 20)]
        assert o["flat2"] == [3.0] * 20 + [1.0 * (r + 1)] * 20 + [3.0] * 10
        assert o["mean_ok"]
        assert o["bcast"] == ([5.0] * 7, [9.0] * 3)
