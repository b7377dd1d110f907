"""Training the ResNet-50 ensemble member (``EnsembleTrainer.train_epoch`` trains every
member of ``EnsembleDetector(['efficientnet_b0', 'resnet50'])``, src/ensemble_trainer.py:158-229,
src/pretrained_detector.py:146-218), fp32, against the oracle restatement of torchvision resnet50
(``oracle/resnet_cpu.py``, run as plain PyTorch fp32 on the GPU with cuDNN/MIOpen off -- test
infrastructure only).

1. Every distinct convolution of the trunk: the training kernels (implicit-GEMM forward with the
   BN-stat partials, data gradient at stride 1 and 2, weight gradient) against torch autograd of
   conv2d on the same fp32 operands.
2. The train-mode trunk: features, every parameter gradient, the BN running buffers and
   ``num_batches_tracked`` after one step, at 4 x 128^2 and 2 x 160^2 frames (layer4's BatchNorms
   then normalise over 64 / 50 values; at 2 x 64^2 -- 8 values -- the reassociated fp32 sums of the
   two implementations already differ by 8e-3 relative on single near-zero features).  Bounds:
   features relative L2 <= ``FEAT_TOL`` and elementwise rtol 1e-3 / atol 1e-4; every gradient
   against the fp64 restatement within ``GRAD_MULT`` x the fp32 oracle's own distance to it (the
   train-mode BatchNorm chain amplifies fp32 rounding to ~1-2 % on the early layers for ANY fp32
   implementation); running buffers rtol 1e-4 / atol 1e-5.  The BatchNorm apply and its backward
   run in torch's centred order, (y - mean) * scale + beta and k1*g + k2*(y - mean) + k3: the folded
   y * scale + shift put layer4's last-block gradients 3-4x further from fp64 than torch fp32 on
   the ensemble step (tools/rn_bn_numerics.py emulates both forms on the CPU: 0.023 -> 0.008).
3. The ensemble step: ``EnsembleDetector`` in train mode, weighted CE, backward -- both members
   receive every gradient, the resnet member's logits and gradients match the oracle trunk + the
   reference head math.
4. bf16 training (round 6, ``compute_dtype='bf16'``): the bottleneck convolutions' bf16 kernels against
   autograd on the same bf16 operands, and the trunk / ensemble step against fp64 within 3x torch's
   own bf16-autocast error.
Parity against torchvision itself is unpinned (not importable here); the oracle is the
restatement pinned by key names / shapes / parameter count (tests/test_resnet.py)."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

import deepfake_amd  # noqa: F401
from deepfake_amd import _lib
from deepfake_amd.pretrained_detector import EnsembleDetector
from deepfake_amd.resnet import ResNet50Trunk
from oracle.resnet_cpu import ResNet50TrunkCPU, resnet_features

pytestmark = pytest.mark.gpu

FEAT_TOL = 1e-4
GRAD_MULT, GRAD_FLOOR = 3.0, 1e-4  # HIP vs fp64 <= max(3 x (torch fp32 vs fp64), 1e-4)

# (Cin, H, Cout, k, stride) of every distinct convolution (torchvision v1.5 Bottleneck) + conv1
SHAPES = [(3, 32, 64, 7, 2), (64, 16, 64, 1, 1), (64, 16, 64, 3, 1), (64, 16, 256, 1, 1), (256, 16, 128, 1, 1),
          (128, 16, 128, 3, 2), (256, 16, 512, 1, 2), (512, 8, 1024, 1, 2), (256, 8, 256, 3, 2),
          (512, 4, 512, 3, 1), (1024, 4, 2048, 1, 2)]


def _rel(a, b):
    return float((a.double() - b.double()).norm() / (b.double().norm() + 1e-30))


@pytest.mark.parametrize("cin,h,cout,k,s", SHAPES)
def test_training_conv_kernels_vs_autograd(cuda, cin, h, cout, k, s):
    lib = _lib.load()
    st = _lib.stream_of(cuda)
    g = torch.Generator().manual_seed(cin * 7 + k)
    n, p = 3, (k - 1) // 2
    x = torch.randn(n, h, h, cin, generator=g).cuda()
    w = (torch.randn(cout, cin, k, k, generator=g) / (k * k * cin) ** 0.5).cuda()
    ho = (h + 2 * p - k) // s + 1
    dy = torch.randn(n, ho, ho, cout, generator=g).cuda()
    xs = (ctypes.c_int64 * 4)(h * h * cin, h * cin, cin, 1)
    rows = lib.dfd_rn_conv_stat_rows(n, ho, ho)
    stats = torch.empty(rows * 2 * cout, device=cuda)
    wp = torch.empty(2 * w.numel(), device=cuda)
    y = torch.empty(n * ho * ho, cout, device=cuda)
    _lib.check(lib.dfd_rn_train_conv_fwd(st, x.data_ptr(), xs, n, h, h, cin, w.data_ptr(), cout, k, k, s, p,
                                         wp.data_ptr(), y.data_ptr(), stats.data_ptr()))
    dx = torch.empty(n * h * h, cin, device=cuda)
    _lib.check(lib.dfd_rn_conv_dgrad(st, dy.data_ptr(), n, h, h, cin, w.data_ptr(), cout, k, k, s, p, wp.data_ptr(),
                                     wp[w.numel():].data_ptr(), dx.data_ptr()))
    slab = torch.empty(64 * w.numel(), device=cuda)
    dw = torch.empty_like(w)
    _lib.check(lib.dfd_rn_conv_wgrad(st, x.data_ptr(), xs, n, h, h, cin, dy.data_ptr(), cout, k, k, s, p,
                                     slab.data_ptr(), slab.numel(), dw.data_ptr()))
    torch.cuda.synchronize()
    with torch.backends.cudnn.flags(enabled=False):
        xr = x.permute(0, 3, 1, 2).clone().requires_grad_(True)
        wr = w.clone().requires_grad_(True)
        yr = F.conv2d(xr, wr, stride=s, padding=p)
        yr.backward(dy.permute(0, 3, 1, 2))
    yref = yr.detach().permute(0, 2, 3, 1).reshape(-1, cout)
    torch.testing.assert_close(y, yref, rtol=1e-4, atol=1e-4)
    # per 64-row tile: (sum, M2 about the tile's own mean) -- the centred BatchNorm partials
    st2 = stats.view(rows, 2, cout).double()
    yt = torch.nn.functional.pad(yref.double(), (0, 0, 0, rows * 64 - yref.shape[0])).view(rows, 64, cout)
    nt = torch.tensor([min(64, yref.shape[0] - 64 * t) for t in range(rows)], dtype=torch.float64, device=cuda)
    ts = yt.sum(1)
    mt = ts / nt[:, None]
    valid = (torch.arange(64, device=cuda)[None, :] < nt[:, None])[:, :, None]
    m2 = (((yt - mt[:, None, :]) ** 2) * valid).sum(1)
    torch.testing.assert_close(st2[:, 0], ts, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(st2[:, 1], m2, rtol=1e-4, atol=1e-4)
    assert _rel(dx, xr.grad.permute(0, 2, 3, 1).reshape(-1, cin)) < 1e-5
    assert _rel(dw, wr.grad) < 1e-5


def _pair(seed, cuda):
    torch.manual_seed(seed)
    t = ResNet50Trunk("fp32").to(cuda).train()
    ref = ResNet50TrunkCPU().to(cuda).train()
    ref.load_state_dict(t.state_dict())
    return t, ref


@pytest.mark.parametrize("n,hw", [(4, 128), (2, 160)])
def test_train_mode_trunk_vs_oracle(cuda, n, hw):
    t, ref = _pair(3, cuda)
    ref64 = ResNet50TrunkCPU().to(cuda).double().train()
    ref64.load_state_dict(t.state_dict())
    g = torch.Generator().manual_seed(hw)
    x = torch.randn(n, 3, hw, hw, generator=g).cuda()
    dfeat = torch.randn(n, 2048, generator=g).cuda() * 1e-2
    feats = t(x)
    feats.backward(dfeat)
    with torch.backends.cudnn.flags(enabled=False):
        fr = resnet_features(ref, x)
        fr.backward(dfeat)
        f64 = resnet_features(ref64, x.double())
        f64.backward(dfeat.double())
    fe = _rel(feats.detach(), fr.detach())
    print(f"{n}x{hw}^2: features rel L2 {fe:.3g}")
    assert fe <= FEAT_TOL, fe
    torch.testing.assert_close(feats.detach(), fr.detach(), rtol=1e-3, atol=1e-4)
    # gradients: a train-mode ResNet-50 at init amplifies fp32 rounding through its 53 BatchNorm
    # backward passes (measured: torch's own fp32 gradients sit 0.3-2.5 % from the fp64 ones on the
    # early layers), so each HIP gradient is held to the fp64 restatement, within a small multiple of
    # the fp32 oracle's own distance to it
    bad, worst = [], []
    r32, r64 = dict(ref.named_parameters()), dict(ref64.named_parameters())
    for name, p in t.named_parameters():
        assert p.grad is not None, name
        e = _rel(p.grad, r64[name].grad)
        e32 = _rel(r32[name].grad, r64[name].grad)
        worst.append((e, e32, name))
        if e > max(GRAD_MULT * e32, GRAD_FLOOR):
            bad.append((name, e, e32))
    worst.sort(reverse=True)
    print(f"{n}x{hw}^2: worst gradient rel errors vs fp64 (HIP, torch fp32): {worst[:6]}")
    assert not bad, bad
    rb = dict(ref.named_buffers())
    for name, b in t.named_buffers():
        if name.endswith("num_batches_tracked"):
            assert int(b) == int(rb[name]) == 1, name
        else:
            torch.testing.assert_close(b, rb[name], rtol=1e-4, atol=1e-5, msg=lambda m: f"{name}: {m}")


def test_no_grad_train_forward_updates_running_stats(cuda):
    t, ref = _pair(5, cuda)
    x = torch.randn(4, 3, 128, 128).cuda()
    with torch.no_grad():
        f = t(x)
        with torch.backends.cudnn.flags(enabled=False):
            fr = resnet_features(ref, x)
    assert _rel(f, fr) <= FEAT_TOL
    rb = dict(ref.named_buffers())
    for name, b in t.named_buffers():
        if not name.endswith("num_batches_tracked"):
            torch.testing.assert_close(b, rb[name], rtol=1e-4, atol=1e-5)


def test_eval_grad_refused(cuda):
    t = ResNet50Trunk("fp32").to(cuda).eval()
    with pytest.raises(NotImplementedError):
        t(torch.randn(1, 3, 64, 64).cuda())  # parameters require grad, eval mode


# ------------------------------------------------------------------ bf16 training (k_rn16.hip)
@pytest.mark.parametrize("cin,h,cout,k,s", [sh for sh in SHAPES if sh[0] % 64 == 0])
def test_bf16_training_conv_kernels_vs_autograd(cuda, cin, h, cout, k, s):
    """The bf16 training convolutions (bf16 operands, fp32 accumulation) against torch autograd of
    conv2d in fp32 on the SAME bf16-rounded operands: forward (and its BN-stat partials), data gradient
    (stride 1 and 2: the transposed gather) and weight gradient.  Bound: relative L2 <= 1e-2 for the
    bf16-rounded outputs (measured ~2-3e-3: one bf16 rounding of each output), 1e-4 for the fp32 weight
    gradient (fp32 accumulation of exact bf16 products, only the summation order differs)."""
    lib = _lib.load()
    st = _lib.stream_of(cuda)
    g = torch.Generator().manual_seed(cin * 7 + k + 1)
    n, p = 3, (k - 1) // 2
    x = torch.randn(n, h, h, cin, generator=g).cuda().bfloat16()
    w = (torch.randn(cout, cin, k, k, generator=g) / (k * k * cin) ** 0.5).cuda()
    ho = (h + 2 * p - k) // s + 1
    dy = torch.randn(n, ho, ho, cout, generator=g).cuda().bfloat16()
    res = torch.randn(n, h, h, cin, generator=g).cuda().bfloat16()
    wf = torch.empty(w.numel(), dtype=torch.bfloat16, device=cuda)
    wd = torch.empty_like(wf)
    _lib.check(lib.dfd_rn16_pack_weights(st, w.data_ptr(), cout, cin, k, wf.data_ptr(), wd.data_ptr()))
    y = torch.empty(n * ho * ho, cout, dtype=torch.bfloat16, device=cuda)
    stats = torch.empty(2048 * cout, device=cuda)
    rows = ctypes.c_int(0)
    _lib.check(lib.dfd_rn16_conv_fwd(st, x.data_ptr(), n, h, h, cin, wf.data_ptr(), cout, k, s, p, y.data_ptr(),
                                     stats.data_ptr(), ctypes.byref(rows)))
    dx = torch.empty(n * h * h, cin, dtype=torch.bfloat16, device=cuda)
    _lib.check(lib.dfd_rn16_conv_dgrad(st, dy.data_ptr(), n, h, h, cin, wd.data_ptr(), cout, k, s, p, res.data_ptr(),
                                       dx.data_ptr()))
    slab = torch.empty(lib.dfd_rn16_conv_wgrad_slab_floats(n, h, h, cin, cout, k, s, p), device=cuda)
    dw = torch.empty_like(w)
    _lib.check(lib.dfd_rn16_conv_wgrad(st, x.data_ptr(), n, h, h, cin, dy.data_ptr(), cout, k, s, p, slab.data_ptr(),
                                       slab.numel(), dw.data_ptr()))
    torch.cuda.synchronize()
    with torch.backends.cudnn.flags(enabled=False):
        xr = x.float().permute(0, 3, 1, 2).clone().requires_grad_(True)
        wr = w.bfloat16().float().clone().requires_grad_(True)
        yr = F.conv2d(xr, wr, stride=s, padding=p)
        yr.backward(dy.float().permute(0, 3, 1, 2))
    yref = yr.detach().permute(0, 2, 3, 1).reshape(-1, cout)
    assert _rel(y.float(), yref) < 1e-2
    # per-workgroup (sum, sum of squares) rows of the rounded outputs, summed: the batch sums
    st2 = stats[: rows.value * 2 * cout].view(rows.value, 2, cout).double().sum(0)
    yb = y.double()
    torch.testing.assert_close(st2[0], yb.sum(0), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(st2[1], (yb * yb).sum(0), rtol=1e-4, atol=1e-3)
    dxref = xr.grad.permute(0, 2, 3, 1).reshape(-1, cin) + res.float().reshape(-1, cin)
    assert _rel(dx.float(), dxref) < 1e-2
    assert _rel(dw, wr.grad) < 1e-4


def _bf16_pair(seed, cuda):
    torch.manual_seed(seed)
    t = ResNet50Trunk("bf16").to(cuda).train()
    refs = {}
    for dt in (torch.float32, torch.float64):
        refs[dt] = ResNet50TrunkCPU().to(cuda).to(dt).train()
        refs[dt].load_state_dict(t.state_dict())
    return t, refs


BF16_K = 3.0  # each HIP bf16 gradient within 3x torch-bf16-autocast's distance to fp64 on the same step


def test_bf16_train_mode_trunk_vs_fp64(cuda):
    """The bf16 train-mode trunk at 4 x 128^2 against the fp64 restatement, each gradient tensor held to
    BF16_K x the error of torch's own bf16 autocast step (the oracle trunk under torch.autocast bf16,
    MIOpen off) against the same fp64 -- a per-tensor bound anchored to fp64, like the B0 224^2 test.
    Features and the running buffers after the step: the same bound.  At this size (layer4's BatchNorms
    normalise 64 values) bf16 rounding amplified through 53 train-mode BatchNorms leaves BOTH bf16 steps
    far from fp64 (measured: features ~0.16 relative, gradients 1.2-1.7), so the test pins "as close as
    torch's own bf16 step" (worst ratio measured 1.14), not an absolute accuracy."""
    t, refs = _bf16_pair(11, cuda)
    ref_ac = ResNet50TrunkCPU().to(cuda).train()
    ref_ac.load_state_dict(t.state_dict())
    g = torch.Generator().manual_seed(128)
    x = torch.randn(4, 3, 128, 128, generator=g).cuda()
    dfeat = torch.randn(4, 2048, generator=g).cuda() * 1e-2
    feats = t(x)
    feats.backward(dfeat)
    with torch.backends.cudnn.flags(enabled=False):
        f64 = resnet_features(refs[torch.float64], x.double())
        f64.backward(dfeat.double())
        with torch.autocast("cuda", dtype=torch.bfloat16):
            fac = resnet_features(ref_ac, x)
        fac.float().backward(dfeat)
    fe, fa = _rel(feats.detach(), f64.detach()), _rel(fac.detach().float(), f64.detach())
    print(f"bf16 trunk: features rel L2 vs fp64 {fe:.3g} (autocast {fa:.3g})")
    assert fe <= max(BF16_K * fa, 1e-3), (fe, fa)
    r64, rac = dict(refs[torch.float64].named_parameters()), dict(ref_ac.named_parameters())
    bad, rows = [], []
    for name, p in t.named_parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all(), name
        e, ea = _rel(p.grad, r64[name].grad), _rel(rac[name].grad, r64[name].grad)
        rows.append((e / max(ea, 1e-12), name, e, ea))
        if e > max(BF16_K * ea, 1e-3):
            bad.append((name, e, ea))
    rows.sort(reverse=True)
    print("bf16 trunk: worst gradient err / autocast err: " +
          "; ".join(f"{n} {q:.2f} ({e:.2e} vs {a:.2e})" for q, n, e, a in rows[:6]))
    assert not bad, bad
    rb, rba = dict(refs[torch.float64].named_buffers()), dict(ref_ac.named_buffers())
    badb = []
    for name, b in t.named_buffers():
        if name.endswith("num_batches_tracked"):
            assert int(b) == 1, name
        else:
            e, ea = _rel(b, rb[name]), _rel(rba[name], rb[name])
            if e > max(BF16_K * ea, 1e-3):
                badb.append((name, e, ea))
    assert not badb, badb


def test_bf16_ensemble_training_step(cuda):
    """EnsembleDetector(compute_dtype='bf16') trains both members in bf16 (the B0 plan and the ResNet-50
    bottlenecks): every parameter of both members receives a finite gradient and the step is
    bit-reproducible."""
    def run():
        torch.manual_seed(0)
        ens = EnsembleDetector(["efficientnet_b0", "resnet50"], pretrained=False, dropout_rate=0.0,
                               compute_dtype="bf16").to(cuda).train()
        x = torch.randn(2, 2, 3, 128, 128, generator=torch.Generator().manual_seed(1)).cuda()
        logits, _ = ens(x)
        loss = F.cross_entropy(logits, torch.tensor([0, 1]).cuda(), weight=torch.tensor([0.7, 1.3]).cuda())
        loss.backward()
        return float(loss), {f"{mi}.{n}": p.grad.clone() for mi, m in enumerate(ens.models)
                             for n, p in m.named_parameters()}
    la, ga = run()
    lb, gb = run()
    assert all(torch.isfinite(v).all() for v in ga.values())
    assert la == lb
    diff = [n for n in ga if not torch.equal(ga[n], gb[n])]
    assert not diff, diff[:8]


def test_ensemble_training_step(cuda):
    """EnsembleTrainer.train_epoch's step (src/ensemble_trainer.py:188-198) on the default ensemble:
    logits = average of the members, weighted CE, backward; both members get every gradient and the
    resnet member matches the oracle trunk + the reference head math."""
    torch.manual_seed(0)
    ens = EnsembleDetector(["efficientnet_b0", "resnet50"], pretrained=False, dropout_rate=0.0).to(cuda).train()
    x = torch.randn(2, 2, 3, 128, 128).cuda()
    y = torch.tensor([0, 1]).cuda()
    w = torch.tensor([0.7, 1.3]).cuda()
    m = ens.models[1]
    refs = {}
    for dt in (torch.float32, torch.float64):
        refs[dt] = ResNet50TrunkCPU().to(cuda).to(dt).train()
        refs[dt].load_state_dict(m.backbone.state_dict())
    logits, _ = ens(x)
    loss = F.cross_entropy(logits, y, weight=w)
    loss.backward()
    for mi, mem in enumerate(ens.models):
        for n, p in mem.named_parameters():
            assert p.grad is not None and torch.isfinite(p.grad).all(), (mi, n)
    # the resnet member alone, recomputed in fp32 and fp64: oracle trunk + reference head, same loss share
    for dt, ref in refs.items():
        sd = {k: v.detach().to(dt) if v.is_floating_point() else v for k, v in m.state_dict().items()}
        with torch.backends.cudnn.flags(enabled=False):
            f = resnet_features(ref, x.reshape(4, 3, 128, 128).to(dt)).view(2, 2, -1)
            hh = torch.relu(f @ sd["temporal_attention.0.weight"].T + sd["temporal_attention.0.bias"])
            a = torch.sigmoid(hh @ sd["temporal_attention.2.weight"].T + sd["temporal_attention.2.bias"]).squeeze(-1)
            a = torch.softmax(a, dim=1)
            gg = (f * a.unsqueeze(-1)).sum(1)
            z = torch.relu(gg @ sd["fc1.weight"].T + sd["fc1.bias"]) @ sd["fc2.weight"].T + sd["fc2.bias"]
            # d loss / d (resnet member logits) = 1/2 d loss / d (averaged logits): the same loss with the
            # efficientnet member's logits held fixed (recovered from the average)
            l0 = logits.detach().to(dt) * 2 - z.detach()
            lr = F.cross_entropy((l0 + z) / 2, y, weight=w.to(dt))
            lr.backward()
    bad = []
    r32, r64 = dict(refs[torch.float32].named_parameters()), dict(refs[torch.float64].named_parameters())
    for n, p in m.backbone.named_parameters():
        e, e32 = _rel(p.grad, r64[n].grad), _rel(r32[n].grad, r64[n].grad)
        if e > max(GRAD_MULT * e32, GRAD_FLOOR):
            bad.append((n, e, e32))
    worst = sorted(((_rel(p.grad, r64[n].grad), _rel(r32[n].grad, r64[n].grad), n)
                    for n, p in m.backbone.named_parameters()), reverse=True)
    print(f"ensemble step: worst gradient rel errors vs fp64 (HIP, torch fp32): {worst[:6]}")
    assert not bad, bad


def test_ensemble_train_step_fused_adamw(cuda):
    """``TrainStep`` on the ensemble (two flat parameter buffers, one per member): the fused clip +
    AdamW step equals ``clip_grad_norm_(ensemble.parameters(), 1.0)`` + ``torch.optim.AdamW`` on the
    same gradients (src/ensemble_trainer.py:146,199-200)."""
    from deepfake_amd.trainer import TrainStep

    torch.manual_seed(1)
    ens = EnsembleDetector(["efficientnet_b0", "resnet50"], pretrained=False, dropout_rate=0.0).to(cuda).train()
    ts = TrainStep(ens, lr=1e-3, weight_decay=1e-5, class_weights=torch.tensor([0.7, 1.3]), max_grad_norm=1.0)
    x = torch.randn(2, 2, 3, 128, 128).cuda()
    y = torch.tensor([1, 0]).cuda()
    params = list(ens.parameters())
    before = [p.detach().clone() for p in params]
    loss, _ = ts.forward_backward(x, y)
    assert torch.isfinite(loss)
    ref = [b.clone().requires_grad_(True) for b in before]
    for rp, p in zip(ref, params):
        rp.grad = p.grad.detach().clone()
    torch.nn.utils.clip_grad_norm_(ref, 1.0)
    opt = torch.optim.AdamW(ref, lr=1e-3, weight_decay=1e-5)
    opt.step()
    ts.sync_grads()
    ts.optimizer.step()
    changed = 0
    for p, rp, b in zip(params, ref, before):
        torch.testing.assert_close(p.detach(), rp.detach(), rtol=1e-5, atol=1e-7)
        changed += int(not torch.equal(p.detach(), b))
    assert changed >= 0.95 * len(params), (changed, len(params))


def test_second_backward_refused_and_cumulative_momentum(cuda):
    """a second backward through the training node (retain_graph=True) raises a clear
    RuntimeError; BatchNorm2d(momentum=None) updates the running buffers as torch's cumulative
    moving average (factor 1 / num_batches_tracked)."""
    t, ref = _pair(7, cuda)
    x = torch.randn(2, 3, 64, 64).cuda()
    f = t(x)
    f.sum().backward(retain_graph=True)
    with pytest.raises(RuntimeError, match="second backward"):
        f.sum().backward()
    # reference in fp64, each buffer within 1e-3 relative L2: at 2 frames of 64^2 the deepest layers
    # normalise 8 rows of activations that carry the trunk's fp32 chain error (measured worst element
    # 6e-5 absolute on 7.2.bn1.running_mean), while a wrong momentum rule -- the default 0.1 instead
    # of the cumulative 1/2 -- would be off by ~the batch means themselves (tens of %)
    t, ref = _pair(8, cuda)
    ref = ref.double()
    for m in list(t.modules()) + list(ref.modules()):
        if isinstance(m, torch.nn.BatchNorm2d):
            m.momentum = None
    for step in range(2):
        xs = torch.randn(2, 3, 64, 64).cuda()
        with torch.no_grad():
            t(xs)
            with torch.backends.cudnn.flags(enabled=False):
                resnet_features(ref, xs.double())
    rb = dict(ref.named_buffers())
    for name, b in t.named_buffers():
        if name.endswith("num_batches_tracked"):
            assert int(b) == int(rb[name]) == 2, name
        else:
            assert _rel(b, rb[name]) <= 1e-3, (name, _rel(b, rb[name]))
