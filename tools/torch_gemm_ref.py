"""Reference timings of torch.matmul (hipBLASLt) on the B0 pointwise shapes, bf16 -- a yardstick for
the hand-written GEMMs (development tool)."""
import torch

F = 256
shapes = []  # (name, M, N, K)
for name, hw, cin, cout in [("b5 proj", 14, 240, 80), ("b6 exp", 14, 80, 480), ("b6 proj", 14, 480, 80),
                            ("b9 exp", 14, 112, 672), ("b9 proj", 14, 672, 112), ("b11 proj", 7, 672, 192),
                            ("b12 exp", 7, 192, 1152), ("b12 proj", 7, 1152, 192), ("b15 proj", 7, 1152, 320),
                            ("b2 exp", 56, 24, 144), ("b4 exp", 28, 40, 240)]:
    shapes.append((name, F * hw * hw, cout, cin))
dev = "cuda"
for name, M, N, K in shapes:
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
    res = []
    for lab, fn in [("fwd", lambda: x @ w.t()), ("dgrad", lambda: dy @ w), ("wgrad", lambda: dy.t() @ x)]:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res.append(f"{lab} {e0.elapsed_time(e1) / 20 * 1e3:6.1f}")
    fl = 2.0 * (M * K + M * N) / 6.3e12 * 1e6
    print(f"{name:10s} {M}x{N}x{K}  floor {fl:5.1f} us  " + "  ".join(res), flush=True)
