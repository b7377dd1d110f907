# torch CPU bf16 autocast of the fp32 oracle step against the fp32 oracle (test_b0_224_gpu bound); CPU only
# usage: python tools/r05/bf16_floor.py b1t2 b4t8
import sys, time, torch
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import test_b0_224_gpu as T
from oracle.detector_cpu import DetectorCPU
from deepfake_amd.weights import deterministic_init_
for case in sys.argv[1:]:
    t0 = time.time()
    ref = T.oracle_step(case)
    x, labels = T._inputs(case)
    m = DetectorCPU(dropout_rate=0.0); deterministic_init_(m, seed=T.SEED); m.train()
    with torch.autocast("cpu", dtype=torch.bfloat16):
        logits, _ = m(x)
    loss = torch.nn.functional.cross_entropy(logits.float(), labels, weight=T.CLASS_W)
    loss.backward()
    grads = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
    try:
        T._bf16_vs_oracle(case, float(loss), grads, "/torch-autocast-bf16")
    except AssertionError as e:
        print("assert:", e)
    print(case, "time", time.time() - t0)
