"""Time the ViT trunk's GEMM shapes (C5: 128 images x 197 tokens = 25,216 rows) on the own LDS-DMA
kernels (k_vgemm.hip; NT products also with the 256- / 128-wide tile forced, "own256" / "own128", and
with the fragment-pipelined K loop, "xp"; the 768-wide ones also on the 64-wide tile, "own64")
against hipBLASLt,
HIP events on the current stream, interleaved rounds.

usage: python tools/vgemm_bench.py [rounds]   -> one JSON line per shape
"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import deepfake_amd  # noqa: E402,F401
from deepfake_amd import _lib  # noqa: E402

M = 128 * 197
# (name, op, N, K, epi): NT C[M][N] = A[M][K] B[N][K]^T; TN W[N][K] = A[M][N]^T B[M][K]
SHAPES = [("qkv fwd", 0, 2304, 768, 1), ("proj fwd", 0, 768, 768, 3), ("fc1 fwd", 0, 3072, 768, 1),
          ("fc2 fwd", 0, 768, 3072, 3), ("fc2 dgrad", 0, 3072, 768, 0), ("fc1 dgrad", 0, 768, 3072, 0),
          ("proj dgrad", 0, 768, 768, 0), ("qkv dgrad", 0, 768, 2304, 0),
          ("fc2 wgrad", 1, 768, 3072, 0), ("fc1 wgrad", 1, 3072, 768, 0), ("proj wgrad", 1, 768, 768, 0),
          ("qkv wgrad", 1, 2304, 768, 0)]


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda:0")
    lib = _lib.load()
    st = _lib.stream_of(dev)
    P = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
    for name, op, N, K, epi in SHAPES:
        if op == 0:
            A = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
            B = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).bfloat16()
            C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            R = torch.randn(M, N, device=dev).bfloat16() if epi & 2 else None
            bias = torch.randn(N, device=dev) if epi & 1 else None
            slab = None
            args = lambda o: (st, o, P(A), P(B), P(C), P(R), P(bias), None, None, M, N, K, epi, None, 0)  # noqa: E731
        else:
            A = (torch.rand(M, N, device=dev) * 2 - 1).bfloat16()
            B = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
            C = torch.empty(N, K, device=dev)
            slab = torch.empty(max(lib.dfd_vgemm_tn_slab_floats(M, N, K), 4 * N * K), device=dev)
            args = lambda o: (st, o, P(A), P(B), P(C), None, None, None, None, M, N, K, 0, P(slab), slab.numel())  # noqa: E731
        arms = (("own", op), ("blaslt", op + 2)) + ((("own256", 4), ("own128", 5), ("xp", 0)) if op == 0 else ())
        if op == 0 and N == 768:
            arms += (("own64", 7),)
        times = {arm: [] for arm, _ in arms}
        for r in range(rounds + 1):
            for arm, o in arms:
                lib.dfd_set_tuning(b"vg_xp", 3 if arm == "xp" else 0)  # the fragment-pipelined K loop
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                _lib.check(lib.dfd_vgemm(*args(o)))
                e0.record()
                for _ in range(10):
                    _lib.check(lib.dfd_vgemm(*args(o)))
                e1.record()
                torch.cuda.synchronize()
                if r:
                    times[arm].append(e0.elapsed_time(e1) / 10 * 1e3)
        flop = 2.0 * M * N * K
        line = {"shape": name, "M": M, "N": N, "K": K}
        for arm, t in times.items():
            t.sort()
            line[arm + "_us"] = round(t[len(t) // 2], 2)
            line[arm + "_tflops"] = round(flop / (t[len(t) // 2] * 1e-6) / 1e12, 1)
        line["own_over_blaslt"] = round(line["own_us"] / line["blaslt_us"], 3)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
