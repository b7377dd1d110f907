"""Fused bf16 attention (k_attn.hip) through the ``dfd_attention`` seam against plain-PyTorch fp32
attention of the same bf16 operands (softmax(scale q k^T) v and its autograd backward).

Bounds (bf16 storage; fp32 softmax statistics; P and dS rounded to bf16 as MFMA operands):
relative L2 error of O <= 1e-2 and of dq / dk / dv <= 2e-2; the log-sum-exp
within 1e-3 absolute.  Token counts: 197 (ViT-B/16 at 224^2), 17 (64^2 images), 256 (the limit)
and 50 (a ragged count inside a 64-token block)."""
import ctypes

import pytest
import torch

from deepfake_amd import _lib

pytestmark = pytest.mark.gpu
D, H, DH = 768, 12, 64


def _ref(qkv, nt, images, scale, dO):
    x = qkv.float().view(images, nt, 3, H, DH).permute(2, 0, 3, 1, 4)  # 3, img, head, nt, dh
    q, k, v = (t.detach().clone().requires_grad_(True) for t in (x[0], x[1], x[2]))
    s = (q @ k.transpose(-1, -2)) * scale
    lse = torch.logsumexp(s, dim=-1)
    p = torch.softmax(s, dim=-1)
    o = p @ v
    o.backward(dO.float().view(images, nt, H, DH).permute(0, 2, 1, 3))
    return o, lse, q.grad, k.grad, v.grad


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-30))


@pytest.mark.parametrize("images,nt", [(6, 197), (4, 17), (3, 256), (5, 50)])
def test_attention_vs_fp32(cuda, images, nt):
    g = torch.Generator(device=cuda).manual_seed(nt * 13 + images)
    rows = images * nt
    qkv = (torch.randn(rows, 3 * D, device=cuda, generator=g) * 1.5).bfloat16()
    dO = torch.randn(rows, D, device=cuda, generator=g).bfloat16()
    O = torch.zeros(rows, D, device=cuda, dtype=torch.bfloat16)
    lse = torch.zeros(images * H, nt, device=cuda)
    dqkv = torch.full((rows, 3 * D), float("nan"), device=cuda, dtype=torch.bfloat16)
    lib = _lib.load()
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    scale = 0.125
    _lib.check(lib.dfd_attention(None, 0, images, H, nt, scale, P(qkv), 3 * D, D, 2 * D, P(O), D, P(lse), None, 0,
                                 None, 0))
    _lib.check(lib.dfd_attention(None, 1, images, H, nt, scale, P(qkv), 3 * D, D, 2 * D, P(O), D, P(lse), P(dO), D,
                                 P(dqkv), 3 * D))
    torch.cuda.synchronize()
    o_ref, lse_ref, dq, dk, dv = _ref(qkv, nt, images, scale, dO)
    o = O.float().view(images, nt, H, DH).permute(0, 2, 1, 3)
    assert _rel(o, o_ref) <= 1e-2, _rel(o, o_ref)
    torch.testing.assert_close(lse.view(images, H, nt), lse_ref.detach(), rtol=0, atol=1e-3)
    d = dqkv.float().view(images, nt, 3, H, DH).permute(2, 0, 3, 1, 4)
    for name, got, ref in (("dq", d[0], dq), ("dk", d[1], dk), ("dv", d[2], dv)):
        e = _rel(got, ref)
        print(f"nt {nt}: {name} rel err {e:.2e}")
        assert e <= 2e-2, (name, e)
