"""Benchmark: face-frames/sec training EfficientNet-B0 224^2, bs=256 frames/GPU (BASELINE.json).

One step = the reference train step (``EnsembleTrainer.train_epoch``,
src/ensemble_trainer.py:182-200) on one synthetic batch of 32 clips x 8 frames x 224x224x3
per GPU: HIP forward (trunk + temporal-attention head, dropout 0.5), weighted CE, HIP
backward, clip_grad_norm_(1.0) + AdamW(lr 1e-4, wd 1e-5) fused -- with every input already
resident in HBM.  N GPUs = N ranks (torch.distributed, RCCL), clips sharded, bucketed
gradient all-reduce overlapped with backward; value = frames of all ranks / max-over-ranks
time.  Rank 0 prints one JSON line.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--dtype bf16|fp32] [--no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import deepfake_amd  # noqa: E402,F401
from deepfake_amd import roofline  # noqa: E402
from deepfake_amd.pretrained_detector import PretrainedBackboneDetector  # noqa: E402
from deepfake_amd.trainer import DataParallelTrainer  # noqa: E402
from deepfake_amd.weights import deterministic_init_  # noqa: E402

CLIPS, T, H, W = 32, 8, 224, 224
METRIC = "face-frames/sec training EfficientNet-B0 224² bs=256/GPU"


def synthetic_batch(rank: int, device):
    """uint8 frames (seed 0+rank) -> /255 -> ImageNet normalise (app.py:1772-1780), NHWC storage
    viewed as (B, T, 3, H, W) like the reference's permute; labels Bernoulli(0.5) seed 1."""
    g = torch.Generator(device=device)
    g.manual_seed(0 + rank)
    u8 = torch.randint(0, 256, (CLIPS, T, H, W, 3), generator=g, device=device, dtype=torch.uint8)
    mean = torch.tensor([0.485, 0.456, 0.406], device=device)
    std = torch.tensor([0.229, 0.224, 0.225], device=device)
    x = ((u8.float() / 255.0) - mean) / std
    x = x.permute(0, 1, 4, 2, 3)  # (B, T, 3, H, W), channels-last strides
    g.manual_seed(1 + 1000 * rank)
    labels = torch.randint(0, 2, (CLIPS,), generator=g, device=device)
    return x, labels


def cpu_baseline(seconds: float = 15.0):
    """The oracle's fp32 PyTorch-CPU restatement of the same step (oracle/detector_cpu.py), on a bounded
    sample: 2 clips x 8 frames of 224^2 per step, timed for ~`seconds`."""
    from oracle import detector_cpu

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    m = detector_cpu.DetectorCPU(dropout_rate=0.5)
    deterministic_init_(m, seed=0)
    m.train()
    opt = torch.optim.AdamW(m.parameters(), lr=1e-4, weight_decay=1e-5)
    x = torch.randn(2, 8, 3, H, W)
    y = torch.tensor([0, 1])
    detector_cpu.train_step(m, x, y, opt)  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        detector_cpu.train_step(m, x, y, opt)
        n += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": round(n * 16 / dt, 3), "unit": "face-frames/s", "cores": threads, "kind": "port",
            "sample": f"{n} steps x 16 frames (2 clips x 8) 224^2, fp32, oracle/detector_cpu.py train_step "
                      f"(AdamW+clip), torch {torch.__version__} threads={threads}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="kernel-selection knob for A/B runs (dfd_set_tuning), e.g. dw_bwd_pre=2")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    if args.tune:
        from deepfake_amd import _lib
        lib = _lib.load()
        for kv in args.tune:
            k, v = kv.split("=", 1)
            lib.dfd_set_tuning(k.encode(), int(v))
    torch.manual_seed(0)
    model = PretrainedBackboneDetector("efficientnet_b0", pretrained=False, num_classes=2, dropout_rate=0.5,
                                       compute_dtype=args.dtype)
    deterministic_init_(model, seed=0)
    model = model.to(dev).train()
    step = DataParallelTrainer(model, lr=1e-4, weight_decay=1e-5, max_grad_norm=1.0,
                               class_weights=torch.tensor([1.0, 1.0]))
    x, labels = synthetic_batch(rank, dev)
    probe = roofline.KernelProbe(model, "dw_fwd", stage=1, block=0)

    for _ in range(args.warmup):
        step(x, labels)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    probe.arm(args.steps)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(x, labels)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    probe.disarm()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed.item())
    loss, _ = step.forward_backward(x, labels)
    finite = bool(torch.isfinite(loss).item())

    frames = CLIPS * T * world * args.steps
    value = frames / elapsed
    if rank == 0:
        rl = probe.report()
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args.cpu_seconds)
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "face-frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic uint8 frames (seeded, on device) -> ImageNet-normalised fp32, random-init weights",
            "config": {"workload": "EfficientNet-B0 detector train step (PretrainedBackboneDetector, temporal "
                                   "attention head, weighted CE, clip 1.0 + AdamW)",
                       "clips_per_gpu": CLIPS, "frames_per_clip": T, "frames_per_gpu": CLIPS * T,
                       "global_frames": CLIPS * T * world, "image": [H, W, 3], "parallelism": f"dp{world}"},
            "loss_finite": finite,
            "roofline": rl,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
