"""Time the late-stage 1x1 GEMM shapes (256 frames, 14x14 / 7x7 maps) on the small-K weight-panel
kernel (k_pw_sk.hip, seam knob pw_sk=1) against the default dispatch (pw_sk=0), interleaved rounds,
HIP events on the current stream, through the dfd_pw_conv seam.

usage: python tools/pw_sk_bench.py [rounds]    -> one JSON line per shape
"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import deepfake_amd  # noqa: E402,F401
from deepfake_amd import _lib  # noqa: E402

# (site, M, N, K, stats, resid)
SHAPES = [("pw_fwd 3.x/4.0", 50176, 480, 80, True, False), ("pwl_dgrad 3.x", 50176, 480, 80, False, False),
          ("pw_fwd 4.1/4.2/5.0", 50176, 672, 112, True, False), ("pwl_dgrad 4.x", 50176, 672, 112, False, False),
          ("pw_fwd 5.x/6.0", 12544, 1152, 192, True, False), ("pwl_dgrad 5.x", 12544, 1152, 192, False, False),
          ("pwl_dgrad 6.0", 12544, 1152, 320, False, False), ("head fwd", 12544, 1280, 320, True, False)]


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda:0")
    lib = _lib.load()
    st = _lib.stream_of(dev)
    for name, M, N, K, stats, resid in SHAPES:
        a = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        r = torch.randn(M, N, device=dev).bfloat16() if resid else None
        sb = torch.zeros(1024 * 2 * N, device=dev) if stats else None
        rows = ctypes.c_int(0)

        def call():
            _lib.check(lib.dfd_pw_conv(st, 1, a.data_ptr(), w.data_ptr(), c.data_ptr(), _lib.ptr(r), M, N, K, 0,
                                       None, None, None, 1, _lib.ptr(sb), ctypes.byref(rows)))

        times = {0: [], 1: []}
        for rd in range(rounds + 1):
            for v in ((0, 1) if rd % 2 == 0 else (1, 0)):
                lib.dfd_set_tuning(b"pw_sk", v)
                call()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    call()
                e1.record()
                torch.cuda.synchronize()
                if rd:
                    times[v].append(e0.elapsed_time(e1) / 20 * 1e3)
        lib.dfd_set_tuning(b"pw_sk", 0)
        alg = 2 * (M * K + M * N + N * K) + (2 * M * N if resid else 0)
        line = {"site": name, "M": M, "N": N, "K": K}
        for v, t in times.items():
            t.sort()
            med = t[len(t) // 2]
            line[("sk" if v else "default") + "_us"] = round(med, 2)
            line[("sk" if v else "default") + "_hbm_frac"] = round(alg / (med * 1e-6) / 8e12, 3)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
