"""torch.ops.dfd.* registration (the modules call operators, the C ABI sits under them).

CPU: every operator is registered with its schema, shape propagation works under FakeTensorMode,
and a CPU tensor is refused (no CPU kernel, no fallback).  GPU: the operators against torch and
against the module paths that use them."""
import numpy as np
import pytest
import torch

import deepfake_amd  # noqa: F401
from deepfake_amd import ops

SCHEMA_BITS = [
    ("b0_trunk_forward", "Tensor(a3!) buffers"),
    ("b0_trunk_backward", "Tensor(a4!) workspace"),
    ("b0_trunk_backward", "Tensor(a5!) grads"),
    ("weighted_cross_entropy", "Tensor? weight"),
    ("adam_step", "Tensor(a0!) params"),
    ("adam_step", "Tensor(a1!) grads"),  # the clipped gradient is written back
    ("grad_norm", "Tensor(a2!) scratch"),
    ("grad_norm", "Tensor(a3!) out"),
    ("collate_frames", "bool to_float"),
]


def test_ops_registered_with_schemas():
    for name in ops.OPS:
        op = getattr(torch.ops.dfd, name)
        assert op.default._schema.name == f"dfd::{name}"
    for name, bit in SCHEMA_BITS:
        assert bit in str(getattr(torch.ops.dfd, name).default._schema), name


def test_fake_tensor_shapes():
    from torch._subclasses.fake_tensor import FakeTensorMode

    with FakeTensorMode():
        logits = torch.empty(4, 2)
        target = torch.empty(4, dtype=torch.long)
        loss, wsum = torch.ops.dfd.weighted_cross_entropy(logits, target, None, -100)
        assert loss.shape == () and wsum.shape == (1,)
        src = torch.empty(5, 8, 8, 3, dtype=torch.uint8)
        sel = torch.empty(6, dtype=torch.long)
        out = torch.ops.dfd.collate_frames(src, sel, [8, 8, 3], True)
        assert out.shape == (6, 8, 8, 3) and out.dtype == torch.float32


def test_cpu_tensors_refused():
    with pytest.raises(NotImplementedError):
        torch.ops.dfd.weighted_cross_entropy(torch.zeros(2, 2), torch.zeros(2, dtype=torch.long), None, -100)


@pytest.mark.gpu
def test_ce_op_matches_torch_and_backprops():
    g = torch.Generator().manual_seed(3)
    logits = torch.randn(16, 2, generator=g).cuda().requires_grad_(True)
    target = torch.randint(0, 2, (16,), generator=g).cuda()
    target[3] = -100
    w = torch.tensor([0.7, 1.3]).cuda()
    loss, wsum = torch.ops.dfd.weighted_cross_entropy(logits, target, w, -100)
    ref_logits = logits.detach().clone().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(ref_logits, target, weight=w, ignore_index=-100)
    torch.testing.assert_close(loss, ref, rtol=1e-5, atol=1e-6)
    assert abs(float(wsum) - float(w[target[target >= 0]].sum())) < 1e-5
    loss.backward()
    ref.backward()
    torch.testing.assert_close(logits.grad, ref_logits.grad, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_collate_op_bit_exact():
    rng = np.random.default_rng(0)
    src = torch.from_numpy(rng.integers(0, 256, (5, 8, 8, 3), dtype=np.uint8)).cuda()
    sel = torch.tensor([4, 0, -1, 2, 2, 1]).cuda()
    out = torch.ops.dfd.collate_frames(src, sel, [8, 8, 3], True)
    ref = torch.zeros(6, 8, 8, 3)
    for i, s in enumerate(sel.tolist()):
        if s >= 0:
            ref[i] = src[s].cpu().float() / 255.0
    assert torch.equal(out.cpu(), ref)
    raw = torch.ops.dfd.collate_frames(src, sel, [8, 8, 3], False)
    assert raw.dtype == torch.uint8 and torch.equal(raw[0], src[4]) and int(raw[2].abs().sum()) == 0


@pytest.mark.gpu
def test_grad_norm_and_adam_ops():
    g = torch.Generator().manual_seed(5)
    p = torch.randn(1000, generator=g).cuda()
    grad = torch.randn(1000, generator=g).cuda() * 3
    out = torch.zeros(2).cuda()
    scratch = torch.empty(1024, dtype=torch.float64).cuda()
    torch.ops.dfd.grad_norm(grad, 1.0, scratch, out)
    n = float(grad.double().norm())
    assert abs(float(out[0]) - n) <= 1e-5 * n
    assert abs(float(out[1]) - min(1.0, 1.0 / (n + 1e-6))) < 1e-6
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    ref_p = p.clone().requires_grad_(True)
    opt = torch.optim.AdamW([ref_p], lr=1e-3, weight_decay=1e-5)
    ref_p.grad = grad * out[1]
    opt.step()
    torch.ops.dfd.adam_step(p, grad, m, v, 1e-3, 0.9, 0.999, 1e-8, 1e-5, 1, 1.0, True, out)
    torch.testing.assert_close(p, ref_p.detach(), rtol=1e-5, atol=1e-7)


@pytest.mark.gpu
def test_opcheck_optimizer_ops():
    """torch.library.opcheck: the declared mutations (incl. the clipped gradient adam_step writes back and
    grad_norm's scratch) match what the kernels write, and the fake registrations agree."""
    g = torch.Generator().manual_seed(7)
    grad = (torch.randn(4096, generator=g) * 3).cuda()
    out = torch.zeros(2).cuda()
    scratch = torch.zeros(1024, dtype=torch.float64).cuda()
    torch.library.opcheck(torch.ops.dfd.grad_norm.default, (grad, 1.0, scratch, out))
    p = torch.randn(4096, generator=g).cuda()
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    torch.ops.dfd.grad_norm(grad, 1.0, scratch, out)
    torch.library.opcheck(torch.ops.dfd.adam_step.default,
                          (p, grad.clone(), m, v, 1e-3, 0.9, 0.999, 1e-8, 1e-5, 1, 1.0, True, out))
    torch.library.opcheck(torch.ops.dfd.adam_step.default,
                          (p, grad.clone(), m, v, 1e-3, 0.9, 0.999, 1e-8, 0.0, 2, 1.0, False, None))
