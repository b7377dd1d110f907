"""Experiment: capture one whole bench train step in a HIP graph (torch.cuda.CUDAGraph) and time
replays against eager steps.  Timing only -- the captured step freezes host scalars (Adam's step
count, the dropout seed), so replays are not a valid training loop yet."""
import sys, time, os, json
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch
import bench
from deepfake_amd.pretrained_detector import PretrainedBackboneDetector
from deepfake_amd.trainer import DataParallelTrainer
from deepfake_amd.weights import deterministic_init_

dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = PretrainedBackboneDetector("efficientnet_b0", pretrained=False, num_classes=2, dropout_rate=0.5, compute_dtype="bf16")
deterministic_init_(model, seed=0)
model = model.to(dev).train()
step = DataParallelTrainer(model, lr=1e-4, weight_decay=1e-5, max_grad_norm=1.0, class_weights=torch.tensor([1.0, 1.0]))
x, labels = bench.synthetic_batch(0, dev)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(5):
        step(x, labels)
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()

def timed(fn, n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3

eager = timed(lambda: step(x, labels), 20)
g = torch.cuda.CUDAGraph()
out = {"eager_ms": eager}
try:
    with torch.cuda.graph(g):
        step(x, labels)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    out["graph_ms"] = timed(g.replay, 20)
    out["eager_ms_after"] = timed(lambda: step(x, labels), 20)
except Exception as e:  # noqa: BLE001
    out["error"] = repr(e)[:500]
print(json.dumps(out))
