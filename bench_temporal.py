"""Throughput of the temporal-aggregation rows of the hot path on one GPU.

Not the headline bench (that is ``bench.py``, EfficientNet-B0); this measures the two other
reference models behind their drop-in modules, one JSON line each:

* ``CNNLSTMHybrid`` (src/models.py:20-85) train step as ``train.py`` runs it
  (``train.py:104-133``: forward, CE, backward, Adam lr 1e-4) on 16-frame clips, synthetic frames
  (seeded uint8 -> /255, channels-last like ``collate_batch_cnn_lstm``), fp32;
  unit: frames/s (clips x 16 per step).
* ``LogicRNNLSTM`` (src/RNNModel.py) train step (forward with lengths, BCE, backward, Adam) on
  (B, 16, 1024) features; unit: sequence-steps/s (B x T per step).

Each line carries a ``cpu_baseline``: the oracle restatement timed on the host cores for a
bounded sample (the reference itself does not travel to the GPU box).

* ``DeepfakeModel`` (src/models.py:222-291, timm ViT-B/16 + SimpleGCN, config C5) train step in
  bf16 on 128 images (16 graphs x 8 nodes); unit: images/s, plus the MFMA fraction.
* ``EnsembleDetector(['efficientnet_b0', 'resnet50'])`` serving forward (eval, bf16) on 32 clips x 8
  uint8 crops; unit: frames/s (SURVEY §8(f)1,4).
* the same ensemble TRAINED (``--model ensemble_train``; ``EnsembleTrainer.train_epoch``'s step,
  src/ensemble_trainer.py:182-200: forward, weighted CE, backward, clip 1.0 + AdamW over both
  members) on 8 clips x 8 frames, fp32 (the ResNet-50 member trains in fp32); unit: frames/s.

    python bench_temporal.py [--model cnnlstm|rnn|vit|both|all] [--clips 64] [--image 224] [--steps K] [--warmup W]
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

import deepfake_amd  # noqa: E402,F401
from deepfake_amd.cnn_lstm import CNNLSTMHybrid  # noqa: E402
from deepfake_amd.optim import FusedAdam  # noqa: E402
from deepfake_amd.rnn import LogicRNNLSTM  # noqa: E402
from deepfake_amd.weights import deterministic_init_  # noqa: E402


def _time(step, steps, warmup):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def _cpu_time(step, seconds):
    step()
    n, t0 = 0, time.perf_counter()
    while True:
        step()
        n += 1
        if time.perf_counter() - t0 >= seconds:
            return (time.perf_counter() - t0) / n, n


def bench_cnnlstm(args, dev):
    B, T, S = args.clips, 16, args.image
    m = CNNLSTMHybrid(3, 256, 2, 2, 0.3)
    deterministic_init_(m, seed=0)
    m = m.to(dev).train()
    opt = FusedAdam(m.parameters(), lr=1e-4)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    u8 = torch.randint(0, 256, (B, T, S, S, 3), generator=g, device=dev, dtype=torch.uint8)
    x = (u8.float() / 255.0).permute(0, 1, 4, 2, 3)  # (B, T, 3, S, S) channels-last strides (train.py:59)
    y = torch.randint(0, 2, (B,), generator=g, device=dev)
    crit = torch.nn.CrossEntropyLoss()

    def step():
        opt.zero_grad(set_to_none=True)
        loss = crit(m(x), y)
        loss.backward()
        opt.step()

    dt = _time(step, args.steps, args.warmup)
    line = {"metric": "frames/sec training CNNLSTMHybrid 16-frame clips", "value": round(B * T / dt, 2),
            "unit": "frames/s", "n_gpus": 1, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True,
            "dtype": "f32", "data": "synthetic uint8 frames (seeded, on device) /255, random-init weights",
            "config": {"workload": "CNNLSTMHybrid train step (forward, CE, backward, Adam lr 1e-4)",
                       "clips": B, "frames_per_clip": T, "image": [S, S, 3]}}
    if not args.no_cpu_baseline:
        from oracle.detector_cpu import CNNLSTMHybridCPU
        torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1))
        ref = CNNLSTMHybridCPU(3, 256, 2, 2, 0.3).train()
        ropt = torch.optim.Adam(ref.parameters(), lr=1e-4)
        xc = torch.rand(2, T, 3, S, S)
        yc = torch.tensor([0, 1])

        def cstep():
            ropt.zero_grad()
            crit(ref(xc), yc).backward()
            ropt.step()

        ct, n = _cpu_time(cstep, args.cpu_seconds)
        line["cpu_baseline"] = {"value": round(2 * T / ct, 3), "unit": "frames/s", "cores": torch.get_num_threads(),
                                "kind": "port", "sample": f"{n} steps x 2 clips x {T} frames {S}^2, fp32 oracle"}
    return line


def bench_rnn(args, dev):
    B, T, F = args.clips, 16, 1024
    m = LogicRNNLSTM(F, 512, 2, 0.5)
    deterministic_init_(m, seed=0)
    m = m.to(dev).train()
    opt = FusedAdam(m.parameters(), lr=1e-4)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    x = torch.randn(B, T, F, generator=g, device=dev)
    lengths = torch.randint(1, T + 1, (B,), generator=g, device=dev)
    tgt = torch.randint(0, 2, (B, 1), generator=g, device=dev).float()

    def step():
        opt.zero_grad(set_to_none=True)
        loss = torch.nn.functional.binary_cross_entropy(m(x, lengths), tgt)
        loss.backward()
        opt.step()

    dt = _time(step, args.steps, args.warmup)
    line = {"metric": "sequence-steps/sec training LogicRNNLSTM", "value": round(B * T / dt, 2),
            "unit": "sequence-steps/s", "n_gpus": 1, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True,
            "dtype": "f32", "data": "synthetic N(0,1) features, random lengths, random-init weights",
            "config": {"workload": "LogicRNNLSTM train step (forward with lengths, BCE, backward, Adam lr 1e-4)",
                       "batch": B, "steps": T, "input_size": F, "hidden": 512, "layers": 2}}
    if not args.no_cpu_baseline:
        from oracle.detector_cpu import LogicRNNLSTMCPU
        torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1))
        ref = LogicRNNLSTMCPU(F, 512, 2, 0.5).train()
        ropt = torch.optim.Adam(ref.parameters(), lr=1e-4)
        xc, lc, tc = x.cpu(), lengths.cpu(), tgt.cpu()

        def cstep():
            ropt.zero_grad()
            torch.nn.functional.binary_cross_entropy(ref(xc, lc), tc).backward()
            ropt.step()

        ct, n = _cpu_time(cstep, args.cpu_seconds)
        line["cpu_baseline"] = {"value": round(B * T / ct, 3), "unit": "sequence-steps/s",
                                "cores": torch.get_num_threads(), "kind": "port",
                                "sample": f"{n} steps of the same batch, fp32 oracle"}
    return line


def bench_vit(args, dev):
    """C5: ``DeepfakeModel`` (src/models.py:222-291, timm ViT-B/16 branch) train step in bf16 on
    128 images = ``--graphs`` x ``--nodes`` face crops with the chain graph of collate_batch
    (train.py:62-100); CE, backward, Adam.  Unit: images/s; ViT-B/16 is 35.1 GFLOP/img forward
    (SURVEY §8(a)), about 3x that for a train step."""
    from deepfake_amd.detector import chain_adjacency
    from deepfake_amd.vit_gcn import DeepfakeModel

    B, N, S = args.graphs, args.nodes, 224
    m = DeepfakeModel(compute_dtype="bf16")
    deterministic_init_(m, seed=0)
    m = m.to(dev).train()
    opt = FusedAdam(m.parameters(), lr=1e-4)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    u8 = torch.randint(0, 256, (B, N, S, S, 3), generator=g, device=dev, dtype=torch.uint8)
    x = (u8.float() / 255.0).permute(0, 1, 4, 2, 3)
    a = torch.from_numpy(chain_adjacency(N)).float().to(dev).expand(B, N, N).contiguous()
    y = torch.randint(0, 2, (B,), generator=g, device=dev)
    crit = torch.nn.CrossEntropyLoss()

    def step():
        opt.zero_grad(set_to_none=True)
        loss = crit(m(x, a), y)
        loss.backward()
        opt.step()

    dt = _time(step, args.steps, args.warmup)
    imgs = B * N
    tflops = 3 * 35.1e9 * imgs / dt / 1e12
    line = {"metric": "images/sec training DeepfakeModel (ViT-B/16 + GCN)", "value": round(imgs / dt, 2),
            "unit": "images/s", "n_gpus": 1, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True,
            "dtype": "bf16", "data": "synthetic uint8 frames (seeded, on device) /255, random-init weights",
            "config": {"workload": "DeepfakeModel train step (ViT-B/16 CLS features -> SimpleGCN -> classifier; CE, "
                                   "backward, Adam lr 1e-4)", "graphs": B, "nodes": N, "images": imgs,
                       "image": [S, S, 3]},
            "mfma": {"achieved_tflops": round(tflops, 1), "peak_tflops": 2500.0, "frac": round(tflops / 2500.0, 4),
                     "flops_per_image": "3 x 35.1 GFLOP (train step ~ 3x forward)"}}
    if not args.no_cpu_baseline:
        from oracle.vit_cpu import DeepfakeModelCPU
        torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1))
        ref = DeepfakeModelCPU().train()
        ropt = torch.optim.Adam(ref.parameters(), lr=1e-4)
        xc = torch.rand(1, 2, 3, S, S)
        ac = torch.from_numpy(chain_adjacency(2)).float().unsqueeze(0)
        yc = torch.tensor([1])

        def cstep():
            ropt.zero_grad()
            crit(ref(xc, ac), yc).backward()
            ropt.step()

        ct, n = _cpu_time(cstep, args.cpu_seconds)
        line["cpu_baseline"] = {"value": round(2 / ct, 3), "unit": "images/s", "cores": torch.get_num_threads(),
                                "kind": "port", "sample": f"{n} steps x 1 graph x 2 nodes {S}^2, fp32 oracle"}
    return line


def bench_ensemble(args, dev):
    """Serving (SURVEY §8(f)1,4): the app's default ``EnsembleDetector(['efficientnet_b0', 'resnet50'])``
    (app.py:661,1597) in eval mode, bf16, on ``--clips`` x 8 uint8 face crops per call (app MAX_FRAMES,
    app.py:2050); forward only.  Unit: frames/s; the B0-only detector is timed beside it."""
    from deepfake_amd.pretrained_detector import EnsembleDetector, PretrainedBackboneDetector

    B, T, S = args.clips, 8, 224
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    u8 = torch.randint(0, 256, (B, T, S, S, 3), generator=g, device=dev, dtype=torch.uint8)
    x = u8.permute(0, 1, 4, 2, 3)  # uint8 crops, normalised inside the first convolution of each member
    res = {}
    for name, m in (("ensemble", EnsembleDetector(["efficientnet_b0", "resnet50"], pretrained=False,
                                                  compute_dtype="bf16")),
                    ("b0", PretrainedBackboneDetector(pretrained=False, compute_dtype="bf16"))):
        m = m.to(dev).eval()

        def step():
            with torch.no_grad():
                m(x)

        res[name] = _time(step, args.steps, args.warmup)
        if name == "b0":  # the fused 7x7-stage MBConv (knob mbconv7; eval launch is barrier-free)
            m.backbone.runtime().set_tuning("mbconv7", 1)
            res["b0_mbconv7"] = _time(step, args.steps, args.warmup)
            m.backbone.runtime().set_tuning("mbconv7", 0)
    dt = res["ensemble"]
    return {"metric": "frames/sec serving EnsembleDetector(efficientnet_b0 + resnet50)", "value": round(B * T / dt, 2),
            "unit": "frames/s", "n_gpus": 1, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True,
            "dtype": "bf16", "data": "synthetic uint8 face crops (seeded, on device), random-init weights",
            "config": {"workload": "EnsembleDetector eval forward (average of both members)", "clips": B,
                       "frames_per_clip": T, "image": [S, S, 3]},
            "b0_only": {"value": round(B * T / res["b0"], 2), "ms_per_step": round(res["b0"] * 1e3, 3)},
            "b0_only_mbconv7": {"value": round(B * T / res["b0_mbconv7"], 2),
                                "ms_per_step": round(res["b0_mbconv7"] * 1e3, 3)}}


def bench_ensemble_train(args, dev, dtype="fp32"):
    """SURVEY §8(f)4 training: the default ensemble's train step (both members, fp32 -- the reference's
    precision -- or bf16: the B0 plan and the ResNet-50 bottlenecks on bf16 MFMA, k_rn16.hip)."""
    from deepfake_amd.pretrained_detector import EnsembleDetector
    from deepfake_amd.trainer import TrainStep

    B, T, S = args.clips, 8, 224
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    x = torch.rand(B, T, 3, S, S, generator=g, device=dev)
    y = torch.randint(0, 2, (B,), generator=g, device=dev)
    ens = EnsembleDetector(["efficientnet_b0", "resnet50"], pretrained=False, compute_dtype=dtype).to(dev).train()
    ts = TrainStep(ens, lr=1e-4, weight_decay=1e-5, class_weights=torch.tensor([0.7, 1.3]), max_grad_norm=1.0)

    def step():
        ts(x, y)

    dt = _time(step, args.steps, args.warmup)
    return {"metric": "frames/sec training EnsembleDetector(efficientnet_b0 + resnet50)", "value": round(B * T / dt, 2),
            "unit": "frames/s", "n_gpus": 1, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True,
            "dtype": "f32" if dtype == "fp32" else dtype, "data": "synthetic U(0,1) frames (seeded, on device), random-init weights",
            "config": {"workload": "EnsembleDetector train step (both members; weighted CE, clip 1.0 + AdamW)",
                       "clips": B, "frames_per_clip": T, "image": [S, S, 3]}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="both", choices=["cnnlstm", "rnn", "vit", "ensemble", "ensemble_train", "both", "all"])
    ap.add_argument("--graphs", type=int, default=16)
    ap.add_argument("--nodes", type=int, default=8)
    ap.add_argument("--clips", type=int, default=64)
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--ens-dtypes", default="fp32,bf16", help="ensemble_train: compute dtypes, one line each")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if args.model in ("rnn", "both", "all"):
        print(json.dumps(bench_rnn(args, dev)), flush=True)
    if args.model in ("cnnlstm", "both", "all"):
        print(json.dumps(bench_cnnlstm(args, dev)), flush=True)
    if args.model in ("vit", "all"):
        print(json.dumps(bench_vit(args, dev)), flush=True)
    if args.model in ("ensemble", "all"):
        args.clips = min(args.clips, 32)
        print(json.dumps(bench_ensemble(args, dev)), flush=True)
    if args.model in ("ensemble_train", "all"):
        args.clips = min(args.clips, 8)
        for dt in args.ens_dtypes.split(","):
            print(json.dumps(bench_ensemble_train(args, dev, dt)), flush=True)


if __name__ == "__main__":
    main()
