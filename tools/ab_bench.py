"""In-process A/B of kernel-selection knobs on the bench step (interleaved, so clock drift cancels).

usage: python tools/ab_bench.py KEY V1 V2 [V3 ...] [--rounds R] [--steps S]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from deepfake_amd import _lib  # noqa: E402
from deepfake_amd.pretrained_detector import PretrainedBackboneDetector  # noqa: E402
from deepfake_amd.trainer import DataParallelTrainer  # noqa: E402
from deepfake_amd.weights import deterministic_init_  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("key")
    ap.add_argument("values", nargs="+", type=int)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "bf16"])
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = PretrainedBackboneDetector("efficientnet_b0", pretrained=False, num_classes=2, dropout_rate=0.5,
                                       compute_dtype=a.dtype)
    deterministic_init_(model, seed=0)
    model = model.to(dev).train()
    step = DataParallelTrainer(model, lr=1e-4, weight_decay=1e-5, max_grad_norm=1.0,
                               class_weights=torch.tensor([1.0, 1.0]))
    x, labels = bench.synthetic_batch(0, dev)
    lib = _lib.load()
    res = {v: [] for v in a.values}
    rt = model.backbone.runtime()  # the knob is per plan (dfd_b0_plan_set_tuning)
    for v in a.values:  # warm every variant
        rt.set_tuning(a.key, v)
        for _ in range(2):
            step(x, labels)
    torch.cuda.synchronize()
    for r in range(a.rounds):
        for v in (a.values if r % 2 == 0 else a.values[::-1]):
            rt.set_tuning(a.key, v)
            step(x, labels)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                step(x, labels)
            torch.cuda.synchronize()
            res[v].append(1e3 * (time.perf_counter() - t0) / a.steps)
    for v in a.values:
        ms = sorted(res[v])
        print(f"{a.key}={v}: median {ms[len(ms) // 2]:.3f} ms/step  min {ms[0]:.3f}  all {[round(m, 3) for m in res[v]]}")


if __name__ == "__main__":
    main()
