"""Bit-identity of the ViT-B/16 trunk across library builds: bf16 features and parameter gradients of one
forward + backward at 8 images (sha256 prefixes).  GPU; usage: python tools/r05/vit_hash.py"""
import hashlib
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from b0_helpers import frames  # noqa: E402
from deepfake_amd.vit_gcn import ViTFeatureExtractor  # noqa: E402
from deepfake_amd.weights import deterministic_init_  # noqa: E402

cuda = torch.device("cuda:0")
fx = ViTFeatureExtractor(compute_dtype="bf16")
deterministic_init_(fx, seed=9)
fx = fx.to(cuda)
x = frames(35, (1, 8, 3, 224, 224))[0].to(cuda)
f = fx(x)
(f * torch.linspace(-1, 1, f.numel(), device=cuda).view_as(f)).sum().backward()
torch.cuda.synchronize()
hf = hashlib.sha256(f.detach().cpu().numpy().tobytes()).hexdigest()[:16]
hg = hashlib.sha256(torch.cat([p.grad.flatten() for p in fx.parameters()]).cpu().numpy().tobytes()).hexdigest()[:16]
print("vit bf16 feats", hf, "grads", hg, flush=True)
