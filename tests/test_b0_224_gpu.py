"""224x224 training-step parity of the HIP EfficientNet-B0 detector -- the map sizes the bench runs.

The depthwise kernels pick their tiles from the feature-map size, so only a 224x224 input reaches
the launches the 256-frame bench step runs: the fused stride-1 backward ``dw_bwd1`` on 8x28 tiles
(blocks.0.0, 1.1), 14x14 tiles (k3/k5 on 28x28 and 14x14 maps) and two stacked 7x7 frames
(stages 5/6); the fused stride-2 backward ``dw_bwd2`` on 8x56 tiles (blocks.1.0 k3, 2.0 k5),
whole 28x28 frames (blocks.3.0) and four stacked 14x14 frames (blocks.5.0); the channel-pair
forwards ``dw_fwd1`` and the remaining stride-2 forwards.  Two batches:

* 1 clip x 2 frames: the smallest batch with a non-trivial temporal softmax (and a partly empty
  four-frame tile);
* 4 clips x 8 frames (32 frames, the reference's clip shape): the >=100K-row layers take the
  streaming 1x1 kernels and the BN-folded expansion backward on the default path, and the 28x28
  stage takes the 64x64 GEMM tile -- the bench's selections.

Each runs on the ``default`` and ``forced`` kernel paths (conftest ``kernel_paths``).  The checker
is the fp32 CPU oracle (``oracle/detector_cpu.py``, pinned by the reference goldens in
``test_oracle_golden.py``; trunk numerics "parity unpinned" at the timm boundary) running the
reference step: ``model(images)`` -> ``CrossEntropyLoss(weight)`` -> ``backward``
(``src/ensemble_trainer.py:188-198``, trunk under autograd at ``src/pretrained_detector.py:116``).

Tolerances: fp32 -- logits and loss rtol 1e-3 / atol 1e-5 (north star); every parameter gradient's
norm within 1e-3 relative and its 64 leading elements within rtol 1e-3 / atol 1e-5 + 1e-3 *
max|leading|; BN running statistics rtol 1e-4.  16-bit steps (bf16 / fp16 storage, fp32
accumulation): loss within 2 % of the fp32 oracle, and a PER-TENSOR gradient bound anchored to fp64
(``_vs_fp64``): every gradient's relative L2 error against the oracle run in float64 must stay within
K x the error torch's own bf16 autocast of the same oracle step makes on that tensor (floor 1e-3) --
the bound scales with how ill-conditioned each tensor is, measured, instead of a count of tensors
allowed outside a fixed tolerance (K per dtype at ``K_VS_AUTOCAST``).
"""
import numpy as np
import pytest
import torch

from b0_helpers import frames
from deepfake_amd.pretrained_detector import PretrainedBackboneDetector
from deepfake_amd.weights import deterministic_init_
from oracle.detector_cpu import DetectorCPU

pytestmark = pytest.mark.gpu

SEED = 21
CASES = {"b1t2": (1, 2), "b4t8": (4, 8)}
CLASS_W = torch.tensor([0.7, 1.3])
_ORACLE = {}


def _inputs(case):
    b, t = CASES[case]
    x = frames(SEED + 1, (b, t, 3, 224, 224))
    # channels-last strides, as app.py:2084-2086 / train.py:59 hand the frames over
    x = x.reshape(b * t, 3, 224, 224).contiguous(memory_format=torch.channels_last).view(b, t, 3, 224, 224)
    labels = torch.tensor([(i * 7 + 1) % 2 for i in range(b)])
    return x, labels


def oracle_step(case):
    """fp32 CPU oracle: forward, weighted CE, backward (cached per case)."""
    if case not in _ORACLE:
        torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
        x, labels = _inputs(case)
        m = DetectorCPU(dropout_rate=0.0)
        deterministic_init_(m, seed=SEED)
        m.train()
        logits, scores = m(x)
        loss = torch.nn.functional.cross_entropy(logits, labels, weight=CLASS_W)
        loss.backward()
        _ORACLE[case] = dict(
            logits=logits.detach(), scores=scores.detach(), loss=float(loss),
            grads={n: p.grad.detach().clone() for n, p in m.named_parameters()},
            bufs={n: b.detach().clone() for n, b in m.named_buffers() if "running" in n})
    return _ORACLE[case]


def hip_step(case, dtype, cuda, loss_scale=1.0):
    """One HIP train step; loss_scale: the loss is multiplied by it before backward and the gradients
    divided by it after (a static loss scale, the fp16 recipe)."""
    x, labels = _inputs(case)
    torch.manual_seed(0)
    det = PretrainedBackboneDetector("efficientnet_b0", pretrained=False, num_classes=2, dropout_rate=0.0,
                                     compute_dtype=dtype)
    deterministic_init_(det, seed=SEED)
    det = det.to(cuda).train()
    logits, scores = det(x.to(cuda))
    loss = torch.nn.functional.cross_entropy(logits, labels.to(cuda), weight=CLASS_W.to(cuda))
    (loss * loss_scale if loss_scale != 1.0 else loss).backward()
    torch.cuda.synchronize()
    grads = {n: p.grad.detach().cpu() / loss_scale for n, p in det.named_parameters()}
    bufs = {n: b.detach().cpu() for n, b in det.named_buffers() if "running" in n}
    return logits.detach().cpu(), scores.detach().cpu(), float(loss), grads, bufs


@pytest.mark.parametrize("case", list(CASES))
def test_train_step_224_fp32(cuda, case, kernel_paths):
    if kernel_paths == "split_dw":
        pytest.skip("the two-kernel depthwise backward is covered at 64x64 (test_b0_parity_gpu.py)")
    ref = oracle_step(case)
    logits, scores, loss, grads, bufs = hip_step(case, "fp32", cuda)
    torch.testing.assert_close(logits, ref["logits"], rtol=1e-3, atol=1e-5)
    torch.testing.assert_close(scores, ref["scores"], rtol=1e-3, atol=1e-5)
    assert abs(loss - ref["loss"]) <= 1e-3 * abs(ref["loss"]) + 1e-5
    assert sorted(grads) == sorted(ref["grads"])
    bad = []
    for n, rg in ref["grads"].items():
        g = grads[n].double().flatten()
        r = rg.double().flatten()
        rn = float(r.norm())
        if abs(float(g.norm()) - rn) > 1e-3 * rn + 1e-6:
            bad.append((n, "norm", float(g.norm()), rn))
        k = min(64, r.numel())
        atol = 1e-5 + 1e-3 * float(r[:k].abs().max())
        if not np.allclose(g[:k].numpy(), r[:k].numpy(), rtol=1e-3, atol=atol):
            bad.append((n, "head", float((g[:k] - r[:k]).abs().max())))
    print(f"{case}/{kernel_paths}: {len(ref['grads'])} gradients, mismatches {len(bad)}: {bad[:12]}")
    assert not bad
    for n, rb in ref["bufs"].items():
        torch.testing.assert_close(bufs[n], rb, rtol=1e-4, atol=1e-6, msg=lambda m: f"{n}: {m}")


# The 16-bit bound, per tensor: rel_err(HIP 16-bit grad, fp64 oracle grad) <= K * max(rel_err(torch bf16
# autocast grad, fp64 oracle grad), 1e-3).  torch's autocast (CPU, same oracle module, same inputs and
# weights) rounds conv inputs / outputs to bf16 like the HIP bf16 step stores its activations, so its
# error on a tensor measures that tensor's conditioning under bf16 rounding; the HIP step must be no
# worse than K times it.  K is stated per dtype; the measured worst ratios are printed by every run and
# recorded in DESIGN.md (round 6).
K_VS_AUTOCAST = {"bf16": 3.0, "fp16": 1.0}
AUTOCAST_FLOOR = 1e-3
FP16_LOSS_SCALE = 1024.0
_F64, _AC = {}, {}


def oracle64_step(case):
    """the oracle step in float64 on the CPU (inputs, weights and every op in double; cached)"""
    if case not in _F64:
        torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
        x, labels = _inputs(case)
        m = DetectorCPU(dropout_rate=0.0)
        deterministic_init_(m, seed=SEED)
        m = m.double().train()
        logits, _ = m(x.double())
        loss = torch.nn.functional.cross_entropy(logits, labels, weight=CLASS_W.double())
        loss.backward()
        _F64[case] = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
    return _F64[case]


def autocast_err(case):
    """{tensor: rel. L2 error vs fp64} of torch's CPU bf16 autocast of the oracle step (cached)"""
    if case not in _AC:
        g64 = oracle64_step(case)
        x, labels = _inputs(case)
        m = DetectorCPU(dropout_rate=0.0)
        deterministic_init_(m, seed=SEED)
        m.train()
        with torch.autocast("cpu", dtype=torch.bfloat16):
            logits, _ = m(x)
        torch.nn.functional.cross_entropy(logits.float(), labels, weight=CLASS_W).backward()
        _AC[case] = {n: float((p.grad.double() - g64[n]).norm()) / (float(g64[n].norm()) + 1e-300)
                     for n, p in m.named_parameters()}
    return _AC[case]


def _vs_fp64(case, dtype, loss, grads, tag=""):
    """the 16-bit step's loss against the fp32 oracle (2 %) and every gradient against the fp64 oracle
    within K_VS_AUTOCAST[dtype] x torch-bf16-autocast's error on that tensor"""
    ref = oracle_step(case)
    assert abs(loss - ref["loss"]) <= 2e-2 * abs(ref["loss"]), (loss, ref["loss"])
    g64, ac = oracle64_step(case), autocast_err(case)
    k = K_VS_AUTOCAST[dtype]
    scale = max(float(g.norm()) for g in g64.values())
    rows, bad = [], []
    for n, r in g64.items():
        rn = float(r.norm())
        # structurally ~zero (a BN shift feeding only a training-mode BN): rounding residue only
        if rn <= 1e-4 * scale:
            continue
        e = float((grads[n].double() - r).norm()) / rn
        anchor = max(ac[n], AUTOCAST_FLOOR)
        rows.append((e / anchor, n, e, ac[n]))
        if e > k * anchor:
            bad.append((n, round(e, 5), round(ac[n], 5)))
    rows.sort(reverse=True)
    print(f"{case}{tag} {dtype}: {len(rows)} gradients; worst err/autocast-err ratios (K = {k}): "
          + "; ".join(f"{n} {q:.3f} ({e:.2e} vs {a:.2e})" for q, n, e, a in rows[:6]))
    assert len(rows) >= 0.85 * len(g64)
    assert not bad, bad


@pytest.mark.parametrize("case", list(CASES))
def test_train_step_224_bf16(cuda, case, kernel_paths):
    if kernel_paths == "split_dw":
        pytest.skip("the two-kernel depthwise backward is covered at 64x64 (test_b0_parity_gpu.py)")
    ref = oracle_step(case)
    logits, _, loss, grads, bufs = hip_step(case, "bf16", cuda)
    torch.testing.assert_close(logits, ref["logits"], rtol=5e-2, atol=5e-2)
    _vs_fp64(case, "bf16", loss, grads, f"/{kernel_paths}")
    for n, rb in ref["bufs"].items():
        torch.testing.assert_close(bufs[n], rb, rtol=2e-2, atol=2e-2, msg=lambda m: f"{n}: {m}")


@pytest.mark.parametrize("case", list(CASES))
def test_train_step_224_fp16(cuda, case):
    """fp16 storage (v_mfma_f32_16x16x32_f16, fp32 accumulation) under a static loss scale, against
    the same fp32 oracle as the bf16 step (default kernel paths: the bf16-only fused kernels fall
    back to the generic 16-bit ones)."""
    ref = oracle_step(case)
    logits, _, loss, grads, bufs = hip_step(case, "fp16", cuda, loss_scale=FP16_LOSS_SCALE)
    torch.testing.assert_close(logits, ref["logits"], rtol=5e-2, atol=5e-2)
    assert all(torch.isfinite(g).all() for g in grads.values())
    _vs_fp64(case, "fp16", loss, grads)
    for n, rb in ref["bufs"].items():
        torch.testing.assert_close(bufs[n], rb, rtol=2e-2, atol=2e-2, msg=lambda m: f"{n}: {m}")


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
def test_step_224_bit_reproducible(cuda, dtype):
    """Two identical 32-frame 224^2 training steps give bit-identical loss, gradients and BN running
    statistics in both 16-bit modes.  This shape reaches the fused projection backward at its
    dispatched hsplit: the first fp16 build of that kernel (SLP-packed BN2 sums) differed run to run
    there while passing every tolerance test at 64^2 (tools/pwl_det)."""
    a = hip_step("b4t8", dtype, cuda, loss_scale=FP16_LOSS_SCALE if dtype == "fp16" else 1.0)
    b = hip_step("b4t8", dtype, cuda, loss_scale=FP16_LOSS_SCALE if dtype == "fp16" else 1.0)
    assert a[2] == b[2]
    assert torch.equal(a[0], b[0])
    diff = [n for n in a[3] if not torch.equal(a[3][n], b[3][n])]
    assert not diff, diff[:8]
    for n in a[4]:
        assert torch.equal(a[4][n], b[4][n]), n


def test_wgrad_stream_bit_identical(cuda):
    """The 1x1 weight gradients on the plan's second stream (plan knob wgrad_stream = 1; off by default)
    give bit-identical results to the single-stream schedule: same kernels, same fixed-order
    reductions; only the overlap changes (a missing event would show up as a race here)."""
    from deepfake_amd import backbone
    prev = dict(backbone.DEFAULT_TUNING)
    try:
        backbone.DEFAULT_TUNING["wgrad_stream"] = 1
        _, _, loss_a, grads_a, bufs_a = hip_step("b4t8", "bf16", cuda)
        backbone.DEFAULT_TUNING["wgrad_stream"] = 0
        _, _, loss_b, grads_b, bufs_b = hip_step("b4t8", "bf16", cuda)
    finally:
        backbone.DEFAULT_TUNING.clear()
        backbone.DEFAULT_TUNING.update(prev)
    assert loss_a == loss_b
    diff = [n for n in grads_a if not torch.equal(grads_a[n], grads_b[n])]
    assert not diff, diff[:10]
    assert all(torch.equal(bufs_a[n], bufs_b[n]) for n in bufs_a)


@pytest.mark.parametrize("knobs", [{"dw_pf": 1}, {"dw_rb": 1}, {"dw_rb": 2}, {"dw_pf": 1, "dw_rb": 3}])
def test_depthwise_schedule_knobs_close(cuda, knobs):
    """Depthwise schedule knobs (all off by default) against the default schedule on the bf16 step:
    dw_pf = 1, the software-pipelined stride-1 backward (its k3 launches run at 2 workgroups per CU,
    so the grid -- and the fixed-order partial sums of dW and the BN1 statistics -- change); dw_rb
    bit 0 / bit 1, two-row strips in the stride-1 forward / backward (same per-output tap order, the
    BN2 / BN1 / dW partial sums in another pixel order).  None is bit-identical; each must agree with
    the default step like two summation orders of the same bf16 chain: loss within 1e-2 relative and
    every gradient tensor cosine >= 0.998, norm within 3 % for the backward-only knobs (the bounds of
    the fused-MBConv comparison, test_mbconv7_gpu.py).  A forward knob perturbs every train-mode BN2
    statistic of the step, whose rounding flips reach every gradient through the 16 blocks' train-
    mode BatchNorms: two bf16 steps then differ by as much as each differs from the fp32 step (round 5:
    dw_rb bit 0 moved the block-3.0 SE reduce gradient norm by 12 % and the attention bias to cosine
    0.955 between the two), so each of the two runs is held to the bf16-vs-fp32-oracle bound of
    test_train_step_224_bf16 instead -- the variant must be as accurate as the default, not equal to
    it.  The forward's arithmetic itself is held bit-identical in eval mode
    (test_forward_knob_eval_bit_identical)."""
    from deepfake_amd import backbone
    prev = dict(backbone.DEFAULT_TUNING)
    try:
        backbone.DEFAULT_TUNING.update(knobs)
        _, _, loss_a, grads_a, _ = hip_step("b4t8", "bf16", cuda)
        for k in knobs:
            backbone.DEFAULT_TUNING[k] = 0
        _, _, loss_b, grads_b, _ = hip_step("b4t8", "bf16", cuda)
    finally:
        backbone.DEFAULT_TUNING.clear()
        backbone.DEFAULT_TUNING.update(prev)
    assert abs(loss_a - loss_b) <= 1e-2 * abs(loss_b)
    if knobs.get("dw_rb", 0) & 1:  # a forward knob: each run against the fp32 oracle
        _vs_fp64("b4t8", "bf16", loss_a, grads_a, f" {knobs}")
        _vs_fp64("b4t8", "bf16", loss_b, grads_b, " (knobs off)")
        return
    scale = max(float(g.double().norm()) for g in grads_b.values())
    bad = []
    for n, gb in grads_b.items():
        a, b = grads_a[n].double().flatten(), gb.double().flatten()
        nb = float(b.norm())
        if nb <= 1e-3 * scale:
            continue  # structurally ~zero: rounding residue on both sides
        cos = float(a @ b) / (float(a.norm()) * nb + 1e-30)
        if cos < 0.998 or abs(float(a.norm()) - nb) > 3e-2 * nb:
            bad.append((n, round(cos, 6), round(float(a.norm()) / nb, 5)))
    print(f"{knobs} vs default: loss {loss_a:.6f} / {loss_b:.6f}, {len(grads_b)} gradients, outside {bad}")
    assert not bad


def _hip_step_u8(u8, labels, cuda):
    """the bf16 step on dense NHWC uint8 crops (the bench's feed, normalised in the stem)"""
    torch.manual_seed(0)
    det = PretrainedBackboneDetector("efficientnet_b0", pretrained=False, num_classes=2, dropout_rate=0.0,
                                     compute_dtype="bf16")
    deterministic_init_(det, seed=SEED)
    det = det.to(cuda).train()
    logits, _ = det(u8.to(cuda).permute(0, 1, 4, 2, 3))
    loss = torch.nn.functional.cross_entropy(logits, labels.to(cuda), weight=CLASS_W.to(cuda))
    loss.backward()
    torch.cuda.synchronize()
    return float(loss), {n: p.grad.detach().cpu() for n, p in det.named_parameters()}


def _fp64_step_u8(u8, labels, cuda):
    """The reference step (``model(images)`` -> weighted CE -> backward, src/ensemble_trainer.py:188-198)
    in fp64 on the oracle module (plain torch on the GPU, MIOpen off), from the same fp32-normalised
    input the stem computes.  Also returns the per-frame gradient of the temporal-attention's first
    pre-activation (``temporal_attention.0`` output): its bias gradient is the sum of those rows."""
    mean = torch.tensor([0.485, 0.456, 0.406], device=cuda)
    std = torch.tensor([0.229, 0.224, 0.225], device=cuda)
    with torch.backends.cudnn.flags(enabled=False):
        m = DetectorCPU(dropout_rate=0.0)
        deterministic_init_(m, seed=SEED)
        m = m.double().to(cuda).train()
        x = (((u8.to(cuda).float() / 255.0) - mean) / std).double().permute(0, 1, 4, 2, 3)
        keep = {}

        def hook(_mod, _inp, out):
            out.retain_grad()
            keep["pre"] = out

        h = m.temporal_attention[0].register_forward_hook(hook)
        logits, _ = m(x)
        loss = torch.nn.functional.cross_entropy(logits, labels.to(cuda), weight=CLASS_W.to(cuda).double())
        loss.backward()
        h.remove()
        grads = {n: p.grad.detach().cpu() for n, p in m.named_parameters()}
        dpre = keep["pre"].grad.detach().cpu()
    del m, x
    torch.cuda.empty_cache()
    return float(loss), grads, dpre


# temporal_attention.0.bias: |difference| / sum_frames |per-frame term| (see the test below)
TA_BIAS_TOL = 5e-2


_FP64 = {}


@pytest.mark.parametrize("knob,on,off", [("stem_occ", 3, 2), ("tail_fin", 7, 0)])
def test_forward_knob_training_close(cuda, knob, on, off):
    """Forward-schedule knobs on the 32-frame bf16 TRAINING step with the uint8 feed (the configuration
    they change), default against the previous form, and each run against the fp64 step:

    * stem_occ = 3 (default): the stem forward at 3 workgroups per CU, 768 BN-stat partial rows (dense
      uint8 frames only), against stem_occ = 2 (1024 rows);
    * tail_fin = 7 (default): the SE excitation's first product split over its channel slices (another
      fp32 summation order of the squeeze . W_reduce product) and the SE-backward BN2 finalize inside
      the excitation launch, and the BN3 / BN1 / conv_head-BN backward finalize inside the apply pass
      (bn_bwd_apply_fin), against tail_fin = 0 (unsplit excitation, separate finalize launches).

    The bound is the forward-knob one of ``test_depthwise_schedule_knobs_close`` (every gradient tensor
    cosine >= 0.98, norm within 10 %) except for ``temporal_attention.0.bias``, which is judged against
    its own conditioning.  That gradient is  db = sum_frames dpre_f,  dpre_f = dL/dpre at frame f, and
    the attention softmax over a clip's T frames makes the per-clip sum of the upstream logit gradients
    zero: db is a small difference of large per-frame terms (their fp64 l1-sum is kappa times |db|,
    measured and printed), so a relative rounding change of the terms -- a 2^-24-relative change of one
    layer's batch statistics, amplified through the 16 train-mode blocks -- moves db by kappa times as
    much.  Judged like STRUCT_ZERO_TOL in test_b0_bench_config_gpu.py: |a - b|, |a - fp64| and
    |b - fp64| each within TA_BIAS_TOL of the conditioning scale S = |sum_f |dpre_f|| (l2 over the 64
    units).  Measured (stem_occ, round 5): kappa 10.8, |3 - 2| / S = 1.4e-2, |each - fp64| / S = 4.0e-2
    (cosines 0.986 between the two, 0.90 of each to fp64: the bf16 step is equally far from fp64 under
    both partitions).  The between-arm bound holds for the shipped summation orders, not for every valid
    one: with another fp32 order of the SE excitation (measured and reverted, profiles/r05/ab_se_tail_r05w.txt)
    blocks.2.1.0's se.conv_reduce gradient sits at 0.71-0.91 of the fp64 norm across the four variants and
    the conv_head BN weight at cosine 0.959-0.986 to fp64 -- no variant systematically closer to fp64."""
    from deepfake_amd import backbone
    g = torch.Generator().manual_seed(5)
    u8 = torch.randint(0, 256, (4, 8, 224, 224, 3), generator=g, dtype=torch.uint8)
    labels = _inputs("b4t8")[1]
    runs = {}
    prev = dict(backbone.DEFAULT_TUNING)
    try:
        for v in (on, off):
            backbone.DEFAULT_TUNING[knob] = v
            runs[v] = _hip_step_u8(u8, labels, cuda)
    finally:
        backbone.DEFAULT_TUNING.clear()
        backbone.DEFAULT_TUNING.update(prev)
    if "u8" not in _FP64:
        _FP64["u8"] = _fp64_step_u8(u8, labels, cuda)
    loss64, ref, dpre = _FP64["u8"]
    (loss_a, grads_a), (loss_b, grads_b) = runs[on], runs[off]
    assert abs(loss_a - loss_b) <= 1e-2 * abs(loss_b)
    assert abs(loss_a - loss64) <= 2e-2 * abs(loss64)
    scale = max(float(t.double().norm()) for t in grads_b.values())
    bad = []
    name = "temporal_attention.0.bias"
    for n, gb in grads_b.items():
        if n == name:
            continue
        a, b = grads_a[n].double().flatten(), gb.double().flatten()
        nb = float(b.norm())
        if nb <= 1e-3 * scale:
            continue  # structurally ~zero: rounding residue on both sides
        cos = float(a @ b) / (float(a.norm()) * nb + 1e-30)
        if cos < 0.98 or abs(float(a.norm()) - nb) > 0.10 * nb:
            bad.append((n, round(cos, 6), round(float(a.norm()) / nb, 5)))
    r = ref[name].double()
    a, b = grads_a[name].double(), grads_b[name].double()
    assert torch.allclose(dpre.sum(dim=(0, 1)), r, rtol=1e-9, atol=1e-12)  # db is the sum of the per-frame rows
    S = float(dpre.abs().sum(dim=(0, 1)).norm())
    kappa = S / float(r.norm())
    e_ab, e_a, e_b = (float((u - v).norm()) / S for u, v in ((a, b), (a, r), (b, r)))
    cos_ab = float(a @ b) / float(a.norm() * b.norm())
    print(f"{knob} {on} vs {off}: loss {loss_a:.6f} / {loss_b:.6f} (fp64 {loss64:.6f}); outside {bad}; {name}: "
          f"cos(on, off) {cos_ab:.4f}, cos(on, fp64) {float(a @ r) / float(a.norm() * r.norm()):.4f}, "
          f"cos(off, fp64) {float(b @ r) / float(b.norm() * r.norm()):.4f}; kappa {kappa:.1f}; "
          f"|on-off|/S {e_ab:.2e}, |on-fp64|/S {e_a:.2e}, |off-fp64|/S {e_b:.2e}")
    assert not bad
    assert max(e_ab, e_a, e_b) <= TA_BIAS_TOL, (e_ab, e_a, e_b)


@pytest.mark.parametrize("knob,on,off", [("dw_rb", 1, 0), ("stem_occ", 3, 2)])
def test_forward_knob_eval_bit_identical(cuda, knob, on, off):
    """Eval mode (running statistics, no batch sums): the two-row forward strips (dw_rb bit 0)
    compute every depthwise output from the same taps in the same order as the one-row strips, and
    the stem forward at 3 workgroups per CU (stem_occ = 3, the default for dense uint8 frames; 2 is the
    previous occupancy) every output pixel with the same MFMA, so the logits are bit-identical.  (In
    training the occupancy changes the BN-stat row partition -- 768 instead of 1024 rows --:
    test_forward_knob_training_close compares the two training steps with each other and with fp64.)"""
    from deepfake_amd import backbone
    x, _ = _inputs("b4t8")
    if knob == "stem_occ":  # the dense-uint8 stem (the bench's feed): uint8 NHWC crops, permuted view
        g = torch.Generator().manual_seed(5)
        x = torch.randint(0, 256, (4, 8, 224, 224, 3), generator=g, dtype=torch.uint8).permute(0, 1, 4, 2, 3)
    outs = []
    prev = dict(backbone.DEFAULT_TUNING)
    try:
        for v in (on, off):
            backbone.DEFAULT_TUNING[knob] = v
            det = PretrainedBackboneDetector("efficientnet_b0", pretrained=False, num_classes=2, dropout_rate=0.0,
                                             compute_dtype="bf16")
            deterministic_init_(det, seed=SEED)
            det = det.to(cuda).eval()
            with torch.no_grad():
                logits, _ = det(x.to(cuda))
            outs.append(logits.float().cpu())
    finally:
        backbone.DEFAULT_TUNING.clear()
        backbone.DEFAULT_TUNING.update(prev)
    assert torch.isfinite(outs[1]).all()
    assert torch.equal(outs[0], outs[1])

