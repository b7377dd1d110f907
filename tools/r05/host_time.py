"""Host enqueue cost of one bench step vs its GPU time (is the step host-bound?).

After a sync (empty queue) the wall time of step() without a sync is the host's enqueue cost; the
synced time of K back-to-back steps / K is the device-bound step time."""
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
for _ in range(5):
    step(x, labels)
torch.cuda.synchronize()
host = []
for _ in range(10):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step(x, labels)
    host.append(time.perf_counter() - t0)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    step(x, labels)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 20
# split of the host time: forward+loss, backward, optimizer
parts = []
for _ in range(5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step.optimizer.zero_grad(set_to_none=True)
    out = model(x)
    loss = step.criterion(out[0], labels)
    t1 = time.perf_counter()
    loss.backward()
    t2 = time.perf_counter()
    step.optimizer.step()
    t3 = time.perf_counter()
    parts.append((t1 - t0, t2 - t1, t3 - t2))
print(json.dumps({"host_enqueue_ms": sorted(host)[len(host) // 2] * 1e3, "device_step_ms": dt * 1e3,
                  "fwd_ms": min(p[0] for p in parts) * 1e3, "bwd_ms": min(p[1] for p in parts) * 1e3,
                  "opt_ms": min(p[2] for p in parts) * 1e3}))
