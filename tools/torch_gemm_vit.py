"""torch.matmul (hipBLASLt) yardstick on the ViT-B/16 GEMM shapes at 128 images (development tool)."""
import torch

M = 128 * 197
dev = "cuda"
for name, N, K in [("qkv", 2304, 768), ("proj", 768, 768), ("fc1", 3072, 768), ("fc2", 768, 3072)]:
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
        us = e0.elapsed_time(e1) / 20 * 1e3
        res.append(f"{lab} {us:7.1f} us {2.0 * M * N * K / us / 1e6:6.0f} TF")
    print(f"{name:5s} {M}x{N}x{K}  " + "  ".join(res), flush=True)
