"""Bit-identity across library builds: one B0 forward + backward (224, bench batch) per dtype, printing a
sha256 of the features and of the flat gradient.  Run once per DFD_HIP_LIB and compare the lines.
GPU; usage: python tools/r05/libhash.py [frames]"""
import hashlib
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import test_pwl_fused_gpu as T  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 256
cuda = torch.device("cuda:0")
for dtype in ("bf16", "fp16"):
    det = T.PretrainedBackboneDetector("efficientnet_b0", pretrained=False, num_classes=2, dropout_rate=0.0,
                                       compute_dtype=dtype)
    T.deterministic_init_(det, seed=T.SEED)
    det = det.to(cuda).train()
    det.ensure_flat()
    rt = det.backbone.runtime()
    rt.set_input_norm("imagenet")
    g = torch.Generator().manual_seed(frames * 7 + 224)
    x = torch.randint(0, 256, (frames, 3, 224, 224), generator=g, dtype=torch.uint8).to(cuda)
    with torch.no_grad():
        feats, (h, ws) = rt.forward(x, det, T.DT[dtype], True)
        gd = torch.Generator(device=cuda).manual_seed(5)
        dfeat = torch.randn(frames, 1280, device=cuda, generator=gd) * (1e-3 if dtype == "bf16" else 32.768)
        grads = torch.zeros_like(det._flat_p)
        rt.backward(h, ws, x, dfeat, det, grads, True, 0, 9)
    torch.cuda.synchronize()
    hf = hashlib.sha256(feats.float().cpu().numpy().tobytes()).hexdigest()[:16]
    hg = hashlib.sha256(grads.cpu().numpy().tobytes()).hexdigest()[:16]
    print(dtype, "feats", hf, "grads", hg, flush=True)
