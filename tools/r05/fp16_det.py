"""fp16 vs bf16: backward determinism (same knob twice) and fused-vs-unfused projection backward, per
tensor cosine; prints the worst tensors.  GPU; usage: python tools/r05/fp16_det.py [frames]"""
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import test_pwl_fused_gpu as T  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 32
cuda = torch.device("cuda:0")
for dtype in ("bf16", "fp16"):
    for knob, seq in (("pwl_fused", (False, False)), ("pwl_fused", (False, True)), ("fold_fused", (False, True))):
        out = T._run(cuda, frames, 224, seq if seq[0] != seq[1] else (False,), knob=knob, dtype=dtype)
        if seq[0] == seq[1]:
            out2 = T._run(cuda, frames, 224, (False,), knob=knob, dtype=dtype)
            a, b = out[False], out2[False]
        else:
            a, b = out[False], out[True]
        rows = []
        for n, ra in a.items():
            rb = b[n]
            rn = float(ra.norm())
            if rn == 0:
                continue
            cos = float(ra @ rb) / (rn * float(rb.norm()) + 1e-30)
            rows.append((cos, n, float((ra - rb).norm()) / rn, rn))
        rows.sort()
        same = all(torch.equal(a[n], b[n]) for n in a)
        print(dtype, knob, seq, "bit-identical" if same else "differs", [(n, round(c, 6), round(e, 5), f"{r:.3g}")
                                                                       for c, n, e, r in rows[:4]], flush=True)
        if seq[0] != seq[1]:
            first = {n: (c, e) for c, n, e, r in rows}
            for blk in ("2.1.1", "2.1.0", "2.0.0"):
                sel = [(n.split(".", 3)[3], round(first[n][1], 5)) for n in first if n.startswith(f"backbone.{blk}.")]
                print("   ", blk, sel, flush=True)
