"""fp16 / bf16 backward determinism with the default kernel selection at the bench shape: the same
forward's backward run twice (and a second forward + backward), compared bitwise per tensor.
GPU; usage: python tools/r05/fp16_det2.py [frames]"""
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from deepfake_amd.pretrained_detector import PretrainedBackboneDetector  # noqa: E402
from deepfake_amd.weights import deterministic_init_  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 256
cuda = torch.device("cuda:0")
DT = {"bf16": 1, "fp16": 2}
for dtype in ("fp16", "bf16"):
    det = PretrainedBackboneDetector("efficientnet_b0", pretrained=False, num_classes=2, dropout_rate=0.0,
                                     compute_dtype=dtype)
    deterministic_init_(det, seed=21)
    det = det.to(cuda).train()
    det.ensure_flat()
    rt = det.backbone.runtime()
    rt.set_input_norm("imagenet")
    g = torch.Generator().manual_seed(3)
    x = torch.randint(0, 256, (frames, 3, 224, 224), generator=g, dtype=torch.uint8).to(cuda)
    gd = torch.Generator(device=cuda).manual_seed(5)
    dfeat = torch.randn(frames, 1280, device=cuda, generator=gd) * (1e-3 if dtype == "bf16" else 32.768)
    po = det.param_offsets()
    runs = []
    for rep in range(3):
        with torch.no_grad():
            if rep != 1:
                feats, (h, ws) = rt.forward(x, det, DT[dtype], True)
            grads = torch.zeros_like(det._flat_p)
            rt.backward(h, ws, x, dfeat, det, grads, True, 0, 9)
        torch.cuda.synchronize()
        runs.append((feats.clone(), {n: grads[po[n]:po[n] + p.numel()].clone() for n, p in det.named_parameters()}))
    for a, b, what in ((0, 1, "same forward, backward twice"), (0, 2, "forward + backward again")):
        fa, ga = runs[a]
        fb, gb = runs[b]
        diff = [(n, float((ga[n] - gb[n]).norm() / (ga[n].norm() + 1e-30))) for n in ga if not torch.equal(ga[n], gb[n])]
        diff.sort(key=lambda t: -t[1])
        print(dtype, frames, what, "features equal" if torch.equal(fa, fb) else "FEATURES DIFFER",
              f"{len(diff)} gradient tensors differ", diff[:6], flush=True)
    del det, ws, runs
    torch.cuda.empty_cache()
