"""ViT-B/16 inference forward at 128 images, bf16: keep_backward 0 (fc1 stores gelu alone) vs 1 (the
training forward's gelu + derivative), interleaved, CUDA-event timed.  GPU; python tools/r05/vit_inf.py"""
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from b0_helpers import frames  # noqa: E402
from deepfake_amd import vit_gcn  # noqa: E402
from deepfake_amd.weights import deterministic_init_  # noqa: E402

cuda = torch.device("cuda:0")
fx = vit_gcn.ViTFeatureExtractor(compute_dtype="bf16")
deterministic_init_(fx, seed=9)
fx = fx.to(cuda)
fx.ensure_flat()
x = vit_gcn._images_arg(frames(35, (1, 128, 3, 224, 224))[0].to(cuda).unsqueeze(1))
named = dict(fx._flat_params)
params = [named[n] for n in fx._names]
dt = vit_gcn._DT["bf16"]


def run(sink):
    return vit_gcn._VitFn.forward(vit_gcn._Ctx(), x, fx, "vit.", sink, dt, fx.depth, *params)


with torch.no_grad():
    a, b = run(None), run(object())
    print("bit-identical", bool(torch.equal(a, b)), flush=True)
    for _ in range(3):
        run(None), run(object())
    res = {0: [], 1: []}
    for _ in range(5):
        for keep, sink in ((0, None), (1, object())):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(5):
                run(sink)
            e1.record()
            torch.cuda.synchronize()
            res[keep].append(e0.elapsed_time(e1) / 5)
    print("ms per 128-image forward: keep_backward 0", [round(v, 3) for v in res[0]], "| 1",
          [round(v, 3) for v in res[1]], flush=True)
