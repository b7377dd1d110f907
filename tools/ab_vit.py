"""A/B of a ViT tuning knob (vit_gemm: bit 0 own weight gradients, bit 1 own linears; vit_wsplit:
M-splits of the library weight gradients) on bench_temporal.py's ViT-B/16 + GCN train step,
interleaved rounds.

usage: python tools/ab_vit.py KEY V1 V2 [...] [--rounds R]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench_temporal  # noqa: E402
from deepfake_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("key")
    ap.add_argument("values", nargs="+", type=int)
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    args = argparse.Namespace(graphs=16, nodes=8, steps=3, warmup=1, no_cpu_baseline=True, clips=64, image=224,
                              cpu_seconds=0)
    lib = _lib.load()
    res = {v: [] for v in a.values}
    for _ in range(a.rounds):
        for v in a.values:
            lib.dfd_set_tuning(a.key.encode(), v)
            line = bench_temporal.bench_vit(args, dev)
            res[v].append(line["ms_per_step"])
    for v, ms in res.items():
        print(json.dumps({a.key: v, "ms_per_step": ms}))


if __name__ == "__main__":
    main()
