"""Benchmark: face-frames/sec training EfficientNet-B0 224^2, bs=256 frames/GPU (BASELINE.json).

One step = the reference train step (``EnsembleTrainer.train_epoch``,
src/ensemble_trainer.py:182-200) on one synthetic batch of 32 clips x 8 frames x 224x224x3
per GPU: HIP forward (trunk + temporal-attention head, dropout 0.5), weighted CE, HIP
backward, clip_grad_norm_(1.0) + AdamW(lr 1e-4, wd 1e-5) fused -- with every input already
resident in HBM.  N GPUs = N ranks (one process per GPU, torch.distributed over RCCL), clips
sharded, bucketed gradient all-reduce overlapped with backward; value = frames of all ranks /
max-over-ranks time.  Rank 0 prints one JSON line.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--dtype fp16|bf16|fp32] [--no-cpu-baseline]

``--gpus N`` without a launcher: this process spawns ``torch.distributed.run`` with N ranks on
127.0.0.1 BEFORE touching the GPU and exits with its status (the driver's own
``torch.distributed.run ... bench.py --gpus N`` arrives with WORLD_SIZE=N and runs directly).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

CLIPS, T, H, W = 32, 8, 224, 224
METRIC = "face-frames/sec training EfficientNet-B0 224² bs=256/GPU"
# algorithmic HBM bytes of one 256-frame bf16/fp16 train step (every conv layer's
# fwd X+Y+W, dgrad dY+W+dX, wgrad X+dY+dW; BN/SiLU/SE assumed fused) -> 2.69 ms floor at 8 TB/s
STEP_BYTES_256 = 21.53e9


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    # fp16 (the default: BASELINE.json configs[1] names "train loop bs=256 fp16"): IEEE half storage on
    # v_mfma_f32_16x16x32_f16 with dynamic loss scaling (TrainStep's DynamicLossScaler: scale, unscale,
    # skip-on-overflow and update all on the device, inside the step); bf16 the same kernels on bf16
    ap.add_argument("--dtype", default="fp16", choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--input", default="uint8", choices=["uint8", "fp32"],
                    help="frames handed to the model: raw uint8 crops (normalised in the stem) or fp32")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pw-sweep", action="store_true",
                    help="skip the per-site timing of the 1x1-conv GEMMs (MFMA utilisation block, N = 1)")
    ap.add_argument("--cpu-steps", type=int, default=10, help="CPU baseline: timed steps of 32 frames, all threads")
    ap.add_argument("--no-dp-exposure", action="store_true", help="skip the comm-off timing pass (N > 1)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend of the N-rank path (nccl = RCCL over xGMI; gloo only for the "
                         "1-GPU rehearsal with DFD_BENCH_DEVICE=0)")
    ap.add_argument("--launch-check", action="store_true",
                    help="launcher/rendezvous self-test on CPU (gloo): ranks report and exit, no GPU use")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="kernel-selection knob of the model's plans for A/B runs (dfd_b0_plan_set_tuning), "
                         "e.g. pwl_fused=0")
    return ap.parse_args()


def spawn_ranks(n: int) -> int:
    """Re-run this script under torch.distributed.run with n ranks (child processes; this process
    never initialises the GPU, so no exec-after-GPU-init hazard)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver
    return subprocess.run(cmd, env=env).returncode


def launch_check(world, rank, local):
    import torch
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo")
    t = torch.tensor([float(rank)])
    if world > 1:
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "rank_sum": float(t.item()),
                          "expected": float(sum(range(world)))}))
    if world > 1:
        dist.destroy_process_group()


def synthetic_batch(rank: int, device, fmt="uint8"):
    """uint8 face crops (seed 0+rank), NHWC storage viewed as (B, T, 3, H, W) like the reference's
    permute; labels Bernoulli(0.5) seed 1.  "uint8": the crops go to the model as they
    come out of the .npz feed and the app's /255 + ImageNet normalisation (app.py:1772-1780) runs in
    the stem kernel (bit-identical, tests/test_serving.py); "fp32": normalised by torch first."""
    import torch

    g = torch.Generator(device=device)
    g.manual_seed(0 + rank)
    u8 = torch.randint(0, 256, (CLIPS, T, H, W, 3), generator=g, device=device, dtype=torch.uint8)
    if fmt == "uint8":
        x = u8
    else:
        mean = torch.tensor([0.485, 0.456, 0.406], device=device)
        std = torch.tensor([0.229, 0.224, 0.225], device=device)
        x = ((u8.float() / 255.0) - mean) / std
    x = x.permute(0, 1, 4, 2, 3)  # (B, T, 3, H, W), channels-last strides
    g.manual_seed(1 + 1000 * rank)
    labels = torch.randint(0, 2, (CLIPS,), generator=g, device=device)
    return x, labels


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def _physical_cores():
    try:
        pairs = set()
        phys = core = None
        for line in open("/proc/cpuinfo"):
            if line.startswith("physical id"):
                phys = line.split(":")[1].strip()
            elif line.startswith("core id"):
                core = line.split(":")[1].strip()
                pairs.add((phys, core))
        return len(pairs) or None
    except OSError:
        return None


def cpu_baseline(steps: int):
    """SURVEY §8(d) CPU baseline: the oracle's fp32 PyTorch-CPU restatement of the same step recipe
    (fwd, weighted CE, backward, clip_grad_norm_(1.0), AdamW; oracle/detector_cpu.py) -- the
    reference's own B0 path cannot run (timm is absent and reference code does not travel).
    bs=32 frames (4 clips x 8) x `steps` timed steps on all threads of this GPU's CPU share, plus
    one timed 32-frame step on 1 thread (the app's TORCH_NUM_THREADS=1 default, app.py:103)."""
    import torch

    from oracle import detector_cpu
    from deepfake_amd.weights import deterministic_init_

    nproc = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", "0")) or nproc
    threads = max(1, min(share, nproc))
    try:  # the CPU affinity this process may use (the GPU lease's share of the host)
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    clips = 4
    torch.manual_seed(0)
    m = detector_cpu.DetectorCPU(dropout_rate=0.5)
    deterministic_init_(m, seed=0)
    m.train()
    opt = torch.optim.AdamW(m.parameters(), lr=1e-4, weight_decay=1e-5)
    x = torch.randn(clips, T, 3, H, W)
    y = torch.tensor([0, 1] * (clips // 2))

    def run(nthreads, n):
        torch.set_num_threads(nthreads)
        detector_cpu.train_step(m, x, y, opt)  # warm-up
        t0 = time.perf_counter()
        for _ in range(n):
            detector_cpu.train_step(m, x, y, opt)
        return n * clips * T / (time.perf_counter() - t0)

    fps = run(threads, steps)
    fps1 = run(1, 1)
    torch.set_num_threads(threads)
    return {"value": round(fps, 3), "unit": "face-frames/s", "cores": threads, "kind": "port",
            "value_1thread": round(fps1, 3),
            "sample": f"{steps} timed steps x 32 frames (4 clips x 8) 224^2 fp32 on {threads} threads + 1 step on "
                      f"1 thread; oracle/detector_cpu.py train_step (weighted CE, clip 1.0, AdamW), torch "
                      f"{torch.__version__}",
            "cpu_model": _cpu_model(), "nproc": nproc, "physical_cores": _physical_cores(),
            "affinity_cpus": affinity, "omp_num_threads": share,
            "threads_note": (f"{threads} threads = the GPU lease's CPU share (OMP_NUM_THREADS={share}, "
                             f"affinity {affinity} CPUs) of a {nproc}-CPU host; not the whole host")}


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus or 1) > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(env_world or "1")
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a {world}-rank run "
                         f"as {args.gpus} GPUs")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launch_check:
        return launch_check(world, rank, local)

    import torch
    import torch.distributed as dist

    import deepfake_amd  # noqa: F401
    from deepfake_amd import roofline
    from deepfake_amd.pretrained_detector import PretrainedBackboneDetector
    from deepfake_amd.trainer import DataParallelTrainer
    from deepfake_amd.weights import deterministic_init_

    # DFD_BENCH_DEVICE pins every rank to one device: the 1-GPU rehearsal of the N-rank path
    # (--backend gloo, since RCCL refuses two ranks on one device); never set by the driver
    dev = torch.device("cuda", int(os.environ.get("DFD_BENCH_DEVICE", local)))
    torch.cuda.set_device(dev)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)

    torch.manual_seed(0)
    model = PretrainedBackboneDetector("efficientnet_b0", pretrained=False, num_classes=2, dropout_rate=0.5,
                                       compute_dtype=args.dtype)
    for kv in args.tune or []:
        k, v = kv.split("=", 1)
        model.backbone.runtime().set_tuning(k, int(v))
    deterministic_init_(model, seed=0)
    model = model.to(dev).train()
    step = DataParallelTrainer(model, lr=1e-4, weight_decay=1e-5, max_grad_norm=1.0,
                               class_weights=torch.tensor([1.0, 1.0]))
    x, labels = synthetic_batch(rank, dev, args.input)
    # the dominant launch of the step: the fused stride-2 depthwise backward of blocks.1.0
    # (dw_bwd2_kernel<f16,3,8,56,14,1> / <bf16,...>, 112x112x96 <- 56x56x96, k_dw_bwd2.hip; the largest single
    # kernel in the rocprof trace)
    probe = roofline.KernelProbe(model, "dw_bwd", stage=1, block=0)

    def timed(n, arm=False):
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        if arm:
            probe.arm(n)
        t0 = time.perf_counter()
        for _ in range(n):
            step(x, labels)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if world > 1:
            dist.barrier()
        if arm:
            probe.disarm()
        el = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
        return float(el.item())

    for _ in range(args.warmup):
        step(x, labels)
    elapsed = timed(args.steps, arm=True)
    loss, _ = step.forward_backward(x, labels)
    finite = bool(torch.isfinite(loss).item())
    # fp16: the dynamic loss scale after the warmup + timed steps, and how many of them were applied
    # (an overflowing step is skipped on the device; skipped steps are still timed)
    scaler_info = (None if step.loss_scaler is None else
                   {"scale": step.loss_scaler.get_scale(), "applied_steps": step.loss_scaler.applied_steps(),
                    "attempted_steps": args.warmup + args.steps})
    step.sync_grads()

    dp = None
    if world > 1:
        nb = len(step.bucket_log)
        local_el = None
        if not args.no_dp_exposure:
            step.comm_enabled = False  # same step, no all-reduce: what the exchange costs on top
            local_el = timed(args.steps)
            step.comm_enabled = True
        ms, ms_local = 1000 * elapsed / args.steps, (1000 * local_el / args.steps if local_el else None)
        dp = {"buckets_per_step": nb, "bucket_elems": step.bucket_elems,
              "grad_bytes": int(model._flat_p.numel() * 4), "ms_per_step_no_allreduce": ms_local and round(ms_local, 3),
              "allreduce_exposed_ms": None if ms_local is None else round(ms - ms_local, 3),
              "backend": dist.get_backend()}

    frames = CLIPS * T * world * args.steps
    value = frames / elapsed
    if rank == 0:
        rl = probe.report()
        es = 2 if args.dtype in ("bf16", "fp16") else 4
        step_bytes = STEP_BYTES_256 * es / 2
        ms_step = 1000 * elapsed / args.steps
        if rl is not None:
            rl["step"] = {"algorithmic_bytes": step_bytes, "achieved": round(step_bytes / (ms_step / 1e3) / 1e9, 1),
                          "frac": round(step_bytes / (ms_step / 1e3) / roofline.HBM_PEAK, 4),
                          "floor_ms": round(step_bytes / roofline.HBM_PEAK * 1e3, 3),
                          "source": "SURVEY.md §8(d) algorithmic bytes per 256-frame step"}
        pw = None
        if world == 1 and not args.no_pw_sweep:  # after the timed region; one extra step per site
            pw = roofline.pointwise_sweep(model, lambda: step(x, labels), H, W, CLIPS * T, es)
            torch.cuda.synchronize()
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args.cpu_steps)
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "face-frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": (f"synthetic uint8 face crops (seeded 0+rank, on device), {args.input} frames into the model "
                     "(uint8: ImageNet normalisation inside the stem kernel), random-init weights"),
            "config": {"workload": "EfficientNet-B0 detector train step (PretrainedBackboneDetector, temporal "
                                   "attention head, weighted CE, clip 1.0 + AdamW)",
                       "clips_per_gpu": CLIPS, "frames_per_clip": T, "frames_per_gpu": CLIPS * T,
                       "global_frames": CLIPS * T * world, "image": [H, W, 3], "parallelism": f"dp{world}"},
            "loss_finite": finite,
            "loss_scaler": scaler_info,
            "roofline": rl,
            "pointwise": pw,
            "dp": dp,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
