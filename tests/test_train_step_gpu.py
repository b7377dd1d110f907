"""The train-step tail the bench runs every step: HIP weighted cross entropy, global-norm clipping
and fused Adam/AdamW, against ``torch`` and against the reference's own ``EnsembleTrainer`` step.

Reference recipe (``src/ensemble_trainer.py:182-200``)::

    optimizer.zero_grad(); outputs, _ = model(images); loss = criterion(outputs, labels)
    loss.backward(); clip_grad_norm_(model.parameters(), max_norm=1.0); optimizer.step()

with ``criterion = nn.CrossEntropyLoss(weight=class_weights)`` (``:358``) and
``optim.AdamW(params, lr, weight_decay)`` (``:146``); ``src/train.py:323`` uses ``optim.Adam``.

* ``WeightedCrossEntropyLoss`` (``k_head.hip`` ce_forward/ce_backward) vs
  ``F.cross_entropy(weight=, ignore_index=)``: loss and dlogits, fp32 tolerance.
* ``FusedAdamW(max_grad_norm=1.0)`` / ``FusedAdam`` vs ``clip_grad_norm_`` + ``torch.optim.AdamW`` /
  ``Adam`` over several steps on identical gradients: parameters, clipped ``.grad``, moments, norm;
  a parameter without a gradient is skipped like torch does.
* ``DynamicLossScaler`` + the fused optimizers (the fp16 step's device-side unscale / skip / update)
  vs ``torch.amp.GradScaler`` around the same torch step, with injected inf / nan gradients.
* ``TrainStep`` on ``EnsembleDetector(['efficientnet_b0'])`` in fp32 vs ``train_step_64.npz`` (the
  reference's ``EnsembleTrainer.train_epoch`` run on one batch, tests/golden/make_golden.py).
* Optimizer checkpoints (CPU): the fused optimizers' ``state_dict`` loads into ``torch.optim.AdamW``
  and back (``src/train.py:365-366,401`` save and resume ``optimizer_state``).
"""
import os

import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from deepfake_amd.flat import FlatModule
from deepfake_amd.losses import WeightedCrossEntropyLoss
from deepfake_amd.optim import FusedAdam, FusedAdamW


class _Flat(FlatModule):
    def __init__(self):
        super().__init__()
        torch.manual_seed(3)
        self.a = nn.Linear(37, 19)
        self.b = nn.Linear(19, 5)
        self.c = nn.Parameter(torch.randn(1000) * 0.1)
        self._flatten()


def _grads(step, shapes, scale):
    g = torch.Generator().manual_seed(1000 + step)
    return [torch.randn(s, generator=g) * scale for s in shapes]


# ----------------------------------------------------------------------------------------- CE
@pytest.mark.gpu
@pytest.mark.parametrize("nc,weighted,ignore", [(2, True, False), (2, True, True), (2, False, False),
                                                (5, True, True)])
def test_weighted_ce_vs_torch(cuda, nc, weighted, ignore):
    g = torch.Generator().manual_seed(nc * 10 + weighted * 2 + ignore)
    B = 37
    logits = torch.randn(B, nc, generator=g) * 3
    labels = torch.randint(0, nc, (B,), generator=g)
    if ignore:
        labels[::5] = -100
    w = torch.rand(nc, generator=g) + 0.25 if weighted else None
    ref_l = logits.clone().requires_grad_(True)
    ref = F.cross_entropy(ref_l, labels, weight=w, ignore_index=-100)
    ref.backward(torch.tensor(0.75))
    crit = WeightedCrossEntropyLoss(weight=w)
    x = logits.to(cuda).requires_grad_(True)
    loss = crit(x, labels.to(cuda))
    loss.backward(torch.tensor(0.75, device=cuda))
    torch.testing.assert_close(loss.cpu(), ref.detach(), rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(x.grad.cpu(), ref_l.grad, rtol=1e-5, atol=1e-7)


# ------------------------------------------------------------------------------- clip + Adam(W)
@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["adamw", "adam"])
@pytest.mark.parametrize("scale", [1e-2, 10.0])  # below / above the clip threshold
@pytest.mark.parametrize("freeze", [False, True])
def test_fused_adam_vs_torch(cuda, kind, scale, freeze):
    m = _Flat().to(cuda)
    ref = _Flat()
    params = list(m.parameters())
    rparams = list(ref.parameters())
    shapes = [p.shape for p in params]
    wd = 1e-2 if kind == "adamw" else 1e-3
    Fused, Torch = (FusedAdamW, torch.optim.AdamW) if kind == "adamw" else (FusedAdam, torch.optim.Adam)
    opt = Fused(params, lr=1e-3, weight_decay=wd, max_grad_norm=1.0)
    topt = Torch(rparams, lr=1e-3, weight_decay=wd)
    for step in range(4):
        gs = _grads(step, shapes, scale)
        # even steps: gradients as views of one flat buffer (what GradSink hands autograd); odd: separate
        flat = torch.cat([gg.flatten() for gg in gs]).to(cuda) if step % 2 == 0 else None
        o = 0
        for i, (p, q, gg) in enumerate(zip(params, rparams, gs)):
            skip = freeze and i == 1 and step < 2  # a.bias has no gradient for two steps, then unfreezes
            dg = flat[o:o + gg.numel()].view(gg.shape) if flat is not None else gg.to(cuda)
            o += gg.numel()
            p.grad = None if skip else dg
            q.grad = None if skip else gg.clone()
        tn = torch.nn.utils.clip_grad_norm_([q for q in rparams if q.grad is not None], max_norm=1.0)
        topt.step()
        opt.step()
        torch.cuda.synchronize()
        torch.testing.assert_close(opt.last_grad_norm.cpu(), tn.float(), rtol=1e-5, atol=1e-6)
        for i, (p, q) in enumerate(zip(params, rparams)):
            torch.testing.assert_close(p.detach().cpu(), q.detach(), rtol=1e-5, atol=1e-7,
                                       msg=lambda s: f"step {step} param {i}: {s}")
            if q.grad is not None:
                torch.testing.assert_close(p.grad.cpu(), q.grad, rtol=1e-5, atol=1e-8)
                st, rst = opt.state[p], topt.state[q]
                torch.testing.assert_close(st["exp_avg"].cpu(), rst["exp_avg"], rtol=1e-5, atol=1e-9)
                torch.testing.assert_close(st["exp_avg_sq"].cpu(), rst["exp_avg_sq"], rtol=1e-5, atol=1e-12)
    sd = opt.state_dict()
    tsd = topt.state_dict()
    for k in tsd["state"]:
        assert float(sd["state"][k]["step"]) == float(tsd["state"][k]["step"])


# ------------------------------------------------------ dynamic loss scaling (the fp16 train step)
@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["adamw", "adam"])
@pytest.mark.parametrize("layout", ["one", "two_runs", "frozen"])
def test_loss_scaled_adam_vs_torch_gradscaler(cuda, kind, layout):
    """DynamicLossScaler + FusedAdam(W) (device-side unscale / clip / skip / update) against
    torch.amp.GradScaler around clip_grad_norm_ + torch.optim.AdamW / Adam, fed the same SCALED
    gradients (the gradient of loss * scale): a non-finite step (step 2) is skipped and halves the
    scale, growth_interval = 2 finite steps double it again; parameters, moments, clipped unscaled
    .grad, scale and the step counts of the checkpoint match.  Layouts: one flat buffer; two
    FlatModules (two runs: ``EnsembleDetector`` has one per member); a parameter that never
    gets a gradient (the reference's ``freeze_backbone``)."""
    import warnings

    from deepfake_amd.optim import DynamicLossScaler
    if layout == "two_runs":
        m1, m2 = _Flat().to(cuda), _Flat().to(cuda)
        params = list(m1.parameters()) + list(m2.parameters())
        rparams = list(_Flat().parameters()) + list(_Flat().parameters())
    else:
        m = _Flat().to(cuda)
        params, rparams = list(m.parameters()), list(_Flat().parameters())
    frozen = {1} if layout == "frozen" else set()
    shapes = [p.shape for p in params]
    Fused, Torch = (FusedAdamW, torch.optim.AdamW) if kind == "adamw" else (FusedAdam, torch.optim.Adam)
    opt = Fused(params, lr=1e-3, weight_decay=1e-2, max_grad_norm=1.0)
    topt = Torch(rparams, lr=1e-3, weight_decay=1e-2)
    sc = DynamicLossScaler(cuda, init_scale=2.0 ** 10, growth_interval=2)
    opt.set_loss_scaler(sc)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        tsc = torch.amp.GradScaler("cpu", init_scale=2.0 ** 10, growth_interval=2)
    for step in range(7):
        tsc.scale(torch.tensor(1.0))  # initialises the reference scaler's state
        s = tsc.get_scale()
        gs = [g * s for g in _grads(step, shapes, 10.0 if step % 3 else 1e-2)]
        if step == 2:
            gs[2].view(-1)[17] = float("inf")
        if step == 4:
            gs[0].view(-1)[0] = float("nan")
        flat = torch.cat([gg.flatten() for gg in gs]).to(cuda)
        o = 0
        for i, (p, q, gg) in enumerate(zip(params, rparams, gs)):
            p.grad = None if i in frozen else flat[o:o + gg.numel()].view(gg.shape)
            o += gg.numel()
            q.grad = None if i in frozen else gg.clone()
        tsc.unscale_(topt)
        torch.nn.utils.clip_grad_norm_([q for q in rparams if q.grad is not None], max_norm=1.0)
        tsc.step(topt)
        tsc.update()
        opt.step()
        torch.cuda.synchronize()
        assert sc.get_scale() == tsc.get_scale(), (step, sc.get_scale(), tsc.get_scale())
        assert sc.found_inf() == (step in (2, 4))
        for i, (p, q) in enumerate(zip(params, rparams)):
            torch.testing.assert_close(p.detach().cpu(), q.detach(), rtol=1e-5, atol=1e-7,
                                       msg=lambda t: f"step {step} param {i}: {t}")
            if i in frozen:
                continue
            if step not in (2, 4):  # torch leaves unscaled non-finite grads; the skipped step leaves them scaled
                torch.testing.assert_close(p.grad.cpu(), q.grad, rtol=1e-5, atol=1e-8)
            st, rst = opt.state[p], topt.state[q]
            torch.testing.assert_close(st["exp_avg"].cpu(), rst["exp_avg"], rtol=1e-5, atol=1e-9)
            torch.testing.assert_close(st["exp_avg_sq"].cpu(), rst["exp_avg_sq"], rtol=1e-5, atol=1e-12)
    assert sc.applied_steps() == 5
    sd, tsd = opt.state_dict(), topt.state_dict()
    for k in tsd["state"]:
        assert float(sd["state"][k]["step"]) == float(tsd["state"][k]["step"]) == 5.0


# -------------------------------------------------------------- reference EnsembleTrainer step
def _structurally_zero(golden_dir):
    """Parameters whose reference gradient is ~0 by construction (a BN shift feeding only a
    training-mode BN): their AdamW delta is the sign of rounding residue, so they carry no signal."""
    g = np.load(os.path.join(golden_dir, "b0_train_64.npz"))
    return {str(n) for n, v in zip(g["g_names"], g["g_norm"]) if float(v) <= 1e-6}


@pytest.mark.gpu
def test_train_step_golden(cuda, golden_dir):
    from deepfake_amd.pretrained_detector import EnsembleDetector
    from deepfake_amd.trainer import TrainStep
    from deepfake_amd.weights import deterministic_init_

    g = np.load(os.path.join(golden_dir, "train_step_64.npz"))
    lr, wd = float(g["lr"]), float(g["wd"])
    torch.manual_seed(0)
    ens = EnsembleDetector(["efficientnet_b0"], pretrained=False, num_classes=2, dropout_rate=0.0,
                           ensemble_method="average", compute_dtype="fp32")
    deterministic_init_(ens, seed=int(g["seed"]))
    ens = ens.to(cuda).train()
    before = {n: p.detach().cpu().clone() for n, p in ens.named_parameters()}
    step = TrainStep(ens, lr=lr, weight_decay=wd, class_weights=torch.tensor([1.0, 1.0]), max_grad_norm=1.0)
    loss, _ = step(torch.from_numpy(g["x"]).to(cuda), torch.from_numpy(g["labels"]).to(cuda))
    torch.cuda.synchronize()
    assert abs(float(loss) - float(g["loss"])) <= 1e-3 * abs(float(g["loss"])) + 1e-5
    zero = _structurally_zero(golden_dir)
    names = [str(n) for n in g["delta_names"]]
    params = dict(ens.named_parameters())
    assert sorted(names) == sorted(params)
    bad, checked, unsat = [], 0, 0
    for i, n in enumerate(names):
        if n.split("models.0.", 1)[-1] in zero:
            continue
        p0 = before[n].double().flatten()
        d = (params[n].detach().cpu().double().flatten() - p0)
        k = min(64, d.numel())
        ref = g["delta_head"][i][:k]
        # AdamW's first step moves each element by -lr*g/(|g|+eps) - lr*wd*p: an element whose
        # gradient is far above eps moves by exactly -lr*sign(g) (+ decay); compare those elements
        decay = -lr * wd * p0[:k].numpy()
        sat = np.abs(ref - decay) >= 0.999 * lr
        unsat += int((~sat).sum())
        checked += int(sat.sum())
        if not np.allclose(d[:k].numpy()[sat], ref[sat], rtol=1e-3, atol=1e-9):
            bad.append((n, "head"))
        if abs(float(d.norm()) - float(g["delta_norm"][i])) > 2e-2 * float(g["delta_norm"][i]) + 1e-9:
            bad.append((n, "norm", float(d.norm()), float(g["delta_norm"][i])))
    print(f"checked {checked} saturated leading elements, skipped {unsat} unsaturated; bad: {bad[:10]}")
    assert checked > 0.9 * (checked + unsat)
    assert not bad


# ------------------------------------------------------------------ optimizer checkpoints (CPU)
@pytest.mark.parametrize("Fused,Torch", [(FusedAdamW, torch.optim.AdamW), (FusedAdam, torch.optim.Adam)])
def test_optimizer_state_dict_roundtrip_torch(Fused, Torch):
    m = _Flat()
    ref = _Flat()
    # torch -> fused: moments and per-parameter steps land in the flat buffers the kernel reads
    topt = Torch(ref.parameters(), lr=1e-3, weight_decay=1e-2)
    for step in range(3):
        for q, gg in zip(ref.parameters(), _grads(step, [q.shape for q in ref.parameters()], 0.1)):
            q.grad = gg
        topt.step()
    opt = Fused(m.parameters(), lr=1e-3, weight_decay=1e-2, max_grad_norm=1.0)
    opt.load_state_dict(topt.state_dict())
    assert opt._steps == [3] * len(list(m.parameters()))
    o = 0
    for q in ref.parameters():
        k = q.numel()
        assert torch.equal(opt._m[o:o + k], topt.state[q]["exp_avg"].flatten())
        assert torch.equal(opt._v[o:o + k], topt.state[q]["exp_avg_sq"].flatten())
        o += k
    for p, q in zip(m.parameters(), ref.parameters()):
        assert opt.state[p]["exp_avg"].data_ptr() != 0
        assert torch.equal(opt.state[p]["exp_avg"], topt.state[q]["exp_avg"])
    # fused -> torch
    sd = opt.state_dict()
    t2 = Torch(_Flat().parameters(), lr=1e-3, weight_decay=1e-2)
    t2.load_state_dict(sd)
    for k, st in t2.state.items():
        assert float(st["step"]) == 3.0
    for (k1, a), (k2, b) in zip(sorted(t2.state_dict()["state"].items()), sorted(topt.state_dict()["state"].items())):
        assert torch.equal(a["exp_avg"], b["exp_avg"]) and torch.equal(a["exp_avg_sq"], b["exp_avg_sq"])
