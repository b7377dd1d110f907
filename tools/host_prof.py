"""Host-side cost of the bench step: per-step enqueue time (no sync) vs GPU time, and a cProfile of
the timed steps (tools/host_prof.py [steps]).  Tells whether the step is launch/host bound."""
import cProfile
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
from deepfake_amd.pretrained_detector import PretrainedBackboneDetector  # noqa: E402
from deepfake_amd.trainer import DataParallelTrainer  # noqa: E402
from deepfake_amd.weights import deterministic_init_  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = PretrainedBackboneDetector("efficientnet_b0", pretrained=False, num_classes=2, dropout_rate=0.5,
                                   compute_dtype="bf16")
deterministic_init_(model, seed=0)
model = model.to(dev).train()
step = DataParallelTrainer(model, lr=1e-4, weight_decay=1e-5, max_grad_norm=1.0, class_weights=torch.tensor([1.0, 1.0]))
x, labels = bench.synthetic_batch(0, dev)
for _ in range(5):
    step(x, labels)
torch.cuda.synchronize()
host = []
for _ in range(n):  # one step at a time from an idle GPU: host enqueue time vs step time
    t0 = time.perf_counter()
    step(x, labels)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    host.append((t1 - t0, t2 - t0))
print("per step (isolated): host enqueue %.3f ms, wall %.3f ms" % (
    1e3 * sum(h for h, _ in host) / n, 1e3 * sum(w for _, w in host) / n))
pr = cProfile.Profile()
torch.cuda.synchronize()
t0 = time.perf_counter()
pr.enable()
for _ in range(n):
    step(x, labels)
pr.disable()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print("pipelined x%d under cProfile: host %.3f ms/step, wall %.3f ms/step" % (n, 1e3 * (t1 - t0) / n, 1e3 * (t2 - t0) / n))
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
