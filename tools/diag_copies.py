"""Which host-side ops enqueue device copies in a bench train step (development diagnostic)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
from deepfake_amd.pretrained_detector import PretrainedBackboneDetector
from deepfake_amd.trainer import DataParallelTrainer
from deepfake_amd.weights import deterministic_init_
from deepfake_amd.optim import _flat_view

dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = PretrainedBackboneDetector("efficientnet_b0", pretrained=False, dropout_rate=0.5, compute_dtype="bf16")
deterministic_init_(m, seed=0)
m = m.to(dev).train()
step = DataParallelTrainer(m, lr=1e-4, weight_decay=1e-5, max_grad_norm=1.0, class_weights=torch.tensor([1.0, 1.0]))
x, y = bench.synthetic_batch(0, dev)
for _ in range(2):
    step(x, y)
torch.cuda.synchronize()
gs = [p.grad for p in m.parameters()]
print("flat view of grads:", _flat_view(gs) is not None, "n params", len(gs))
from torch.profiler import profile, ProfilerActivity
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    step(x, y)
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="count", row_limit=25))
print("copy-like events:")
for e in prof.key_averages():
    k = e.key.lower()
    if "copy" in k or "memcpy" in k or "memset" in k:
        print(f"  {e.key[:80]:80s} count {e.count}")
ev = prof.events()
names = [e.name for e in ev]
for i, e in enumerate(ev):
    if "memcpy" in e.name.lower() or "copybuffer" in e.name.lower():
        ctx = [x.name[:40] for x in ev[max(0, i - 3):i]]
        print("  context:", ctx, "->", e.name[:60])
        break
