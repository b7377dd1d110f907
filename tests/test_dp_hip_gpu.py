"""``DataParallelTrainer`` on the REAL HIP detector: two ranks on the one GPU of the box (gloo carries
the all-reduce -- RCCL refuses two ranks per device -- so this is the N-rank code path of
``bench.py --gpus N`` with the transport swapped, not a scaling measurement).

SURVEY §8(e): "the DP gradient must equal the mean of the per-shard single-process gradients".
Each rank builds the HIP ``PretrainedBackboneDetector`` (fp32, dropout 0) from a DIFFERENT seed (the
constructor's broadcast must align them), takes its own clips, runs ``forward_backward`` +
``sync_grads`` (the bucketed all-reduce fired from inside the segmented native backward), and then,
with rank 0's weights, the single-process HIP gradient of every rank's shard.  Checked:

* every ``p.grad`` after ``sync_grads`` equals the mean over ranks of the single-process gradients
  (rtol 1e-5: the same kernels, only the loss scaling and the sum order differ);
* buckets are launched head -> stem (descending flat offsets) and cover every parameter once;
* BatchNorm running statistics stay local: each rank's equal that rank's single-process run and
  differ between ranks (the reference has no SyncBN).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B_PER_RANK, T, HW = 2, 2, 64
CLASS_W = [0.7, 1.3]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard(rank):
    g = torch.Generator().manual_seed(500 + rank)
    x = torch.randint(0, 256, (B_PER_RANK, T, HW, HW, 3), generator=g, dtype=torch.uint8)
    y = torch.tensor([(rank + i) % 2 for i in range(B_PER_RANK)])
    return x, y


def _model(seed, dev):
    from deepfake_amd.pretrained_detector import PretrainedBackboneDetector
    from deepfake_amd.weights import deterministic_init_

    m = PretrainedBackboneDetector(pretrained=False, dropout_rate=0.0, compute_dtype="fp32")
    deterministic_init_(m, seed=seed)
    return m.to(dev).train()


def _worker(rank, world, port, q):
    import sys

    sys.path.insert(0, REPO)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import deepfake_amd  # noqa: F401
    from deepfake_amd.losses import WeightedCrossEntropyLoss
    from deepfake_amd.trainer import DataParallelTrainer, TrainStep

    dev = torch.device("cuda:0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = {}
        m = _model(seed=10 + rank, dev=dev)  # different init per rank: the broadcast aligns them
        tr = DataParallelTrainer(m, bucket_elems=1 << 19, class_weights=torch.tensor(CLASS_W, device=dev))
        w0 = {n: p.detach().clone() for n, p in m.named_parameters()}
        x, y = _shard(rank)
        xd = x.to(dev).permute(0, 1, 4, 2, 3)
        tr.forward_backward(xd, y.to(dev))
        tr.sync_grads()
        torch.cuda.synchronize()
        out["grads"] = {n: p.grad.detach().cpu().numpy().copy() for n, p in m.named_parameters()}
        out["buckets"] = list(tr.bucket_log)
        out["flat_numel"] = int(m._flat_p.numel())
        out["bufs"] = {n: b.detach().cpu().numpy().copy() for n, b in m.named_buffers() if "running" in n}
        # single-process gradients of every shard, from the broadcast (rank 0) weights
        for r in range(world):
            ref = _model(seed=10, dev=dev)
            with torch.no_grad():
                for n, p in ref.named_parameters():
                    p.copy_(w0[n])
            st = TrainStep(ref, class_weights=torch.tensor(CLASS_W, device=dev),
                           criterion=WeightedCrossEntropyLoss(weight=torch.tensor(CLASS_W, device=dev)))
            xr, yr = _shard(r)
            st.forward_backward(xr.to(dev).permute(0, 1, 4, 2, 3), yr.to(dev))
            torch.cuda.synchronize()
            out[f"single{r}"] = {n: p.grad.detach().cpu().numpy().copy() for n, p in ref.named_parameters()}
            out[f"single_bufs{r}"] = {n: b.detach().cpu().numpy().copy() for n, b in ref.named_buffers()
                                      if "running" in n}
            del ref, st
        out["w0_rank0_seed"] = all(torch.equal(w0[n].cpu(), p.detach().cpu())
                                   for n, p in _model(seed=10, dev=dev).named_parameters())
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_dp_trainer_hip_detector_two_ranks(cuda):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    env_prev = os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=280) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
        if env_prev is None:
            os.environ.pop("HSA_ENABLE_IPC_MODE_LEGACY", None)
    for p in procs:
        assert p.exitcode == 0
    r0 = res[0]
    names = list(r0["grads"])
    scale = max(float(np.linalg.norm(g)) for g in r0["single0"].values())
    bad = []
    for r in range(world):
        o = res[r]
        assert o["w0_rank0_seed"], "rank weights were not broadcast from rank 0"
        for n in names:
            mean = (r0["single0"][n].astype(np.float64) + r0["single1"][n].astype(np.float64)) / world
            got = o["grads"][n].astype(np.float64)
            if not np.allclose(got, mean, rtol=1e-5, atol=1e-7 * scale):
                bad.append((r, n, float(np.abs(got - mean).max()), float(np.abs(mean).max())))
        # buckets: head first, then down the trunk; together they cover the flat gradient once
        los = [lo for lo, _ in o["buckets"]]
        assert los == sorted(los, reverse=True), o["buckets"]
        cov = sorted(o["buckets"])
        assert cov[0][0] == 0 and cov[-1][1] == o["flat_numel"], cov
        assert all(a[1] == b[0] for a, b in zip(cov, cov[1:])), cov
        assert len(o["buckets"]) >= 2
        # BatchNorm statistics stay local: this rank's equal its own single-process run
        for n, v in o["bufs"].items():
            np.testing.assert_allclose(v, r0[f"single_bufs{r}"][n], rtol=1e-5, atol=1e-7, err_msg=n)
    assert not bad, bad[:10]
    differ = [n for n in res[0]["bufs"] if not np.allclose(res[0]["bufs"][n], res[1]["bufs"][n])]
    assert len(differ) >= 0.9 * len(res[0]["bufs"])
