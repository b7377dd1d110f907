"""Which knob makes the fp16 backward non-deterministic: backward twice per knob setting, count the
gradient tensors that differ bitwise.  GPU; usage: python tools/r05/fp16_det3.py [frames]"""
import sys

import torch

sys.path.insert(0, ".")
from deepfake_amd.pretrained_detector import PretrainedBackboneDetector  # noqa: E402
from deepfake_amd.weights import deterministic_init_  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 32
cuda = torch.device("cuda:0")
SETS = [{}, {"pwl_fused": 0}, {"fold_fused": 0}, {"pwl_fused": 0, "fold_fused": 0}, {"tail_fin": 0},
        {"stream_min_rows": 1 << 40}, {"dw_pf": 0}, {"dw_rb": 0}, {"wgrad_stream": 0}]
for dtype, code in (("fp16", 2), ("bf16", 1)):
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
    for st in SETS:
        for k, v in st.items():
            rt.set_tuning(k, v)
        res = []
        with torch.no_grad():
            feats, (h, ws) = rt.forward(x, det, code, True)
            for rep in range(2):
                grads = torch.zeros_like(det._flat_p)
                rt.backward(h, ws, x, dfeat, det, grads, True, 0, 9)
                torch.cuda.synchronize()
                res.append(grads.clone())
        nd = [n for n, p in det.named_parameters()
              if not torch.equal(res[0][po[n]:po[n] + p.numel()], res[1][po[n]:po[n] + p.numel()])]
        print(dtype, frames, st, f"{len(nd)} tensors differ", nd[:5], flush=True)
        # reset the knobs this set touched to the runtime defaults
        for k in st:
            rt.set_tuning(k, -(1 << 63))
            rt.tuning.pop(k, None)
    del det, ws
    torch.cuda.empty_cache()
