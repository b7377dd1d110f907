"""Drop-in ``DeepfakeModel`` / ``ViTFeatureExtractor`` / ``SimpleGCN`` on MI355X
(src/models.py:88-107, 199-291; config C5: ViT-B/16, 16 nodes per clip, trained by
``train.py:104-133``).

Same constructor arguments and ``state_dict`` keys as the reference with timm present:
``vit.vit.{cls_token, pos_embed, patch_embed.proj.*, blocks.{i}.{norm1, attn.qkv, attn.proj,
norm2, mlp.fc1, mlp.fc2}.*, norm.*}``, ``gcn.fc{1,2}.*``, ``classifier.{0,3}.*``, and the same
``forward(images (B, N, 3, H, W), A_norm (B, N, N)) -> logits (B, num_classes)``.

The ViT trunk runs behind ``dfd_vit_forward/backward`` (``csrc/vit.cpp``: MFMA GEMMs with fused
bias/residual/GELU, batched attention GEMMs, LayerNorm and softmax kernels) in bf16 storage /
fp32 accumulation by default (``compute_dtype='fp32'`` for exact-fp32 parity runs); the
SimpleGCN + mean + classifier head runs in fp32 behind ``dfd_gcn_head_forward/backward``.
Parameters live in one flat fp32 buffer and gradients land in one flat tensor.  Dropout uses the
library's counter hash (same distribution as torch's, different stream).

Refused, as the reference would need the network for them: ``pretrained_vit=True`` and the
``clip`` / ``dinov2`` backbones (HF hub downloads, ``models.py:110-197``).
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn as nn

from . import _lib
from .flat import FlatModule, GradSink

EMBED, DEPTH, MLP, PATCH = 768, 12, 3072, 16
_DT = {"fp32": 0, "bf16": 1}


class _Attn(nn.Module):
    def __init__(self):
        super().__init__()
        self.qkv = nn.Linear(EMBED, 3 * EMBED)
        self.proj = nn.Linear(EMBED, EMBED)


class _Mlp(nn.Module):
    def __init__(self):
        super().__init__()
        self.fc1 = nn.Linear(EMBED, MLP)
        self.fc2 = nn.Linear(MLP, EMBED)


class _Block(nn.Module):
    def __init__(self):
        super().__init__()
        self.norm1 = nn.LayerNorm(EMBED, eps=1e-6)
        self.attn = _Attn()
        self.norm2 = nn.LayerNorm(EMBED, eps=1e-6)
        self.mlp = _Mlp()


class _PatchEmbed(nn.Module):
    def __init__(self):
        super().__init__()
        self.proj = nn.Conv2d(3, EMBED, kernel_size=PATCH, stride=PATCH)


class VisionTransformerParams(nn.Module):
    """Parameters of timm ``vit_base_patch16_224`` (num_classes=0), timm's names; compute is HIP."""

    def __init__(self, depth=DEPTH):
        super().__init__()
        self.num_features = EMBED
        self.depth = depth
        self.patch_embed = _PatchEmbed()
        self.cls_token = nn.Parameter(torch.zeros(1, 1, EMBED))
        self.pos_embed = nn.Parameter(torch.zeros(1, 197, EMBED))
        self.blocks = nn.Sequential(*[_Block() for _ in range(depth)])
        self.norm = nn.LayerNorm(EMBED, eps=1e-6)


class _VitHolder(nn.Module):
    def __init__(self, depth):
        super().__init__()
        self.vit = VisionTransformerParams(depth)
        self.out_dim = EMBED


class SimpleGCN(nn.Module):
    """``SimpleGCN`` (src/models.py:199-219) parameters; its math runs fused with the node mean
    and classifier in ``dfd_gcn_head_forward`` (DeepfakeModel.forward)."""

    def __init__(self, in_dim, hid_dim=256, out_dim=128, dropout=0.3):
        super().__init__()
        self.fc1 = nn.Linear(in_dim, hid_dim)
        self.fc2 = nn.Linear(hid_dim, out_dim)
        self.dropout = nn.Dropout(dropout)

    def forward(self, H, A_norm):  # pragma: no cover - exercised through DeepfakeModel
        raise NotImplementedError("SimpleGCN runs fused inside DeepfakeModel.forward on MI355X")


def _ptrs(tensors) -> ctypes.Array:
    arr = (ctypes.c_void_p * len(tensors))()
    for i, t in enumerate(tensors):
        arr[i] = t.data_ptr()
    return arr


def _images_arg(images: torch.Tensor):
    _lib.require_hip(images, "images")
    if images.dim() != 5 or images.shape[2] != 3:
        raise ValueError(f"expected (B, N, 3, H, W), got {tuple(images.shape)}")
    if images.dtype != torch.float32:
        images = images.float()
    return images


class _VitFn(torch.autograd.Function):
    """images (B, N, 3, H, W) -> CLS features (B*N, 768); gradients of the ViT parameters."""

    @staticmethod
    def forward(ctx, images, owner, prefix, sink, dtype, depth, *params):
        lib = _lib.load()
        B, N, _, H, W = images.shape
        dev = images.device
        work = torch.empty(int(lib.dfd_vit_work_bytes(dtype, depth, B * N, H, W)), dtype=torch.uint8, device=dev)
        feats = torch.empty(B * N, EMBED, dtype=torch.float32, device=dev)
        xs = (ctypes.c_int64 * 5)(*images.stride())
        # no gradient sink: an inference call (the fc1 epilogue skips the GELU derivative)
        _lib.check(lib.dfd_vit_forward_ex(_lib.stream_of(dev), dtype, depth, B * N, N, H, W, images.data_ptr(), xs,
                                          _ptrs(params), work.data_ptr(), feats.data_ptr(), 0 if sink is None else 1))
        ctx.owner, ctx.prefix, ctx.sink, ctx.dtype, ctx.depth = owner, prefix, sink, dtype, depth
        ctx.dims = (B * N, H, W)
        ctx.work = work
        ctx.params = params
        return feats

    @staticmethod
    def backward(ctx, dfeats):
        lib = _lib.load()
        I, H, W = ctx.dims
        dev = dfeats.device
        scratch = torch.empty(int(lib.dfd_vit_scratch_bytes(ctx.dtype, ctx.depth, I, H, W)), dtype=torch.uint8,
                              device=dev)
        names = [n for n in ctx.owner._names if n.startswith(ctx.prefix)]
        gviews = ctx.sink.views(names)
        _lib.check(lib.dfd_vit_backward(_lib.stream_of(dev), ctx.dtype, ctx.depth, I, H, W, _ptrs(ctx.params),
                                        ctx.work.data_ptr(), scratch.data_ptr(), dfeats.contiguous().data_ptr(),
                                        _ptrs(gviews)))
        ctx.work = None
        return (None, None, None, None, None, None, *gviews)


class _HeadFn(torch.autograd.Function):
    """feats (B*N, 768), A_norm (B, N, N) -> logits; gradients of the head and of feats."""

    @staticmethod
    def forward(ctx, feats, a_norm, owner, sink, dims, training, seed, p, *params):
        lib = _lib.load()
        B, N, Dv, hid, out, C = dims
        dev = feats.device
        work = torch.empty(int(lib.dfd_gcn_head_work_floats(*dims)), dtype=torch.float32, device=dev)
        logits = torch.empty(B, C, dtype=torch.float32, device=dev)
        _lib.check(lib.dfd_gcn_head_forward(_lib.stream_of(dev), *dims, feats.data_ptr(), a_norm.data_ptr(),
                                            _ptrs(params), work.data_ptr(), 1 if training else 0, seed, p,
                                            logits.data_ptr()))
        ctx.owner, ctx.sink, ctx.dims, ctx.training, ctx.seed, ctx.p = owner, sink, dims, training, seed, p
        ctx.work, ctx.a_norm, ctx.params = work, a_norm, params
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        lib = _lib.load()
        dev = dlogits.device
        B, N, Dv = ctx.dims[0], ctx.dims[1], ctx.dims[2]
        scratch = torch.empty(int(lib.dfd_gcn_head_scratch_floats(*ctx.dims)), dtype=torch.float32, device=dev)
        names = [n for n in ctx.owner._names if n.startswith(("gcn.", "classifier."))]
        gviews = ctx.sink.views(names)
        dfeats = torch.empty(B * N, Dv, dtype=torch.float32, device=dev)
        _lib.check(lib.dfd_gcn_head_backward(_lib.stream_of(dev), *ctx.dims, ctx.a_norm.data_ptr(), _ptrs(ctx.params),
                                             ctx.work.data_ptr(), scratch.data_ptr(), 1 if ctx.training else 0,
                                             ctx.seed, ctx.p, dlogits.contiguous().float().data_ptr(), _ptrs(gviews),
                                             dfeats.data_ptr()))
        ctx.work = None
        return (dfeats, None, None, None, None, None, None, None, *gviews)


class DeepfakeModel(FlatModule):
    """``DeepfakeModel`` (src/models.py:222-291), timm-ViT branch, on MI355X."""

    def __init__(self, vit_out=768, gcn_hid=256, gcn_out=128, num_classes=2, pretrained_vit=False,
                 vit_model_name="vit_base_patch16_224", vit_pretrained_path=None, backbone: str = "timm_vit",
                 clip_model_name: str = "openai/clip-vit-base-patch32", clip_pretrained: bool = True,
                 dinov2_model_name: str = "facebook/dinov2-base", dinov2_pretrained: bool = True,
                 compute_dtype: str = "bf16", depth: int = DEPTH):
        super().__init__()
        backbone = (backbone or "timm_vit").lower()
        if backbone not in ("timm_vit", "vit", "timm"):
            raise NotImplementedError(f"backbone {backbone!r} needs a Hugging Face hub download; only the timm ViT "
                                      f"branch runs on the MI355X path")
        if vit_model_name != "vit_base_patch16_224":
            raise NotImplementedError(f"only vit_base_patch16_224 is implemented (got {vit_model_name!r})")
        if pretrained_vit:
            raise RuntimeError("pretrained_vit=True is a network fetch (timm hub); unavailable offline")
        if int(vit_out) != EMBED:
            raise NotImplementedError("vit_proj is Identity only for vit_out=768")
        if compute_dtype not in _DT:
            raise ValueError("compute_dtype must be 'bf16' or 'fp32'")
        self.compute_dtype = compute_dtype
        self.depth = depth
        self.vit = _VitHolder(depth)
        self.vit_proj = nn.Identity()
        self.gcn = SimpleGCN(in_dim=vit_out, hid_dim=gcn_hid, out_dim=gcn_out)
        self.classifier = nn.Sequential(nn.Linear(gcn_out, 64), nn.ReLU(), nn.Dropout(0.3),
                                        nn.Linear(64, num_classes))
        self.gcn_hid, self.gcn_out, self.num_classes = gcn_hid, gcn_out, num_classes
        if vit_pretrained_path is not None:
            self._load_vit(vit_pretrained_path)
        self._flatten()

    def _load_vit(self, path):
        """``vit_pretrained_path`` (models.py:256-271): a state dict (optionally under model /
        state_dict / model_state) for the ViT; loaded with the non-executing loader."""
        try:
            state = torch.load(path, map_location="cpu", weights_only=True)
            if isinstance(state, dict) and ("model" in state or "state_dict" in state or "model_state" in state):
                sd = state.get("model", state.get("state_dict", state.get("model_state", state)))
            else:
                sd = state
            try:
                self.vit.load_state_dict(sd)
            except Exception:
                sd2 = {k.replace("base_model.encoder.", ""): v for k, v in sd.items()}
                self.vit.load_state_dict(sd2, strict=False)
            print(f"Loaded ViT pretrained weights from {path}")
        except Exception as e:  # the reference prints and continues (models.py:270-271)
            print(f"Warning: failed to load ViT weights from {path}: {e}")

    def _on_flatten(self) -> None:
        self._names = [n for n, _ in self._flat_params]

    def forward(self, images: torch.Tensor, A_norm: torch.Tensor) -> torch.Tensor:
        self.ensure_flat()
        images = _images_arg(images)
        B, N = images.shape[0], images.shape[1]
        a = A_norm.to(device=images.device, dtype=torch.float32).contiguous()
        if tuple(a.shape) != (B, N, N):
            raise ValueError(f"A_norm must be (B, N, N) = {(B, N, N)}, got {tuple(a.shape)}")
        named = dict(self._flat_params)
        vit_params = [named[n] for n in self._names if n.startswith("vit.")]
        head_params = [named[n] for n in self._names if n.startswith(("gcn.", "classifier."))]
        training = self.training
        p = float(self.gcn.dropout.p) if training else 0.0
        if training and float(self.classifier[2].p) != p:
            raise NotImplementedError("gcn.dropout and classifier[2] must share one dropout rate")
        seed = int(torch.randint(0, 2**62, (1,)).item()) if p > 0 else 0
        dims = (B, N, EMBED, self.gcn_hid, self.gcn_out, self.num_classes)
        need_grad = torch.is_grad_enabled() and any(q.requires_grad for q in self.parameters())
        sink = GradSink(self) if need_grad else None
        dt = _DT[self.compute_dtype]
        if not need_grad:
            with torch.no_grad():
                feats = _VitFn.forward(_Ctx(), images, self, "vit.", None, dt, self.depth, *vit_params)
                return _HeadFn.forward(_Ctx(), feats, a, self, None, dims, training, seed, p, *head_params)
        feats = _VitFn.apply(images, self, "vit.", sink, dt, self.depth, *vit_params)
        return _HeadFn.apply(feats, a, self, sink, dims, training, seed, p, *head_params)


class ViTFeatureExtractor(FlatModule):
    """``ViTFeatureExtractor`` (src/models.py:88-107) with timm present: ``forward(x (B, 3, H, W))
    -> (B, 768)`` CLS features after the final norm."""

    def __init__(self, model_name="vit_base_patch16_224", pretrained=False, out_dim=768, compute_dtype="bf16",
                 depth=DEPTH):
        super().__init__()
        if model_name != "vit_base_patch16_224":
            raise NotImplementedError(f"only vit_base_patch16_224 is implemented (got {model_name!r})")
        if pretrained:
            raise RuntimeError("pretrained=True is a network fetch (timm hub); unavailable offline")
        self.compute_dtype = compute_dtype
        self.depth = depth
        self.vit = VisionTransformerParams(depth)
        self.out_dim = EMBED
        self._flatten()

    def _on_flatten(self) -> None:
        self._names = [n for n, _ in self._flat_params]

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        self.ensure_flat()
        if x.dim() != 4:
            raise ValueError(f"expected (B, 3, H, W), got {tuple(x.shape)}")
        images = _images_arg(x.unsqueeze(1))
        named = dict(self._flat_params)
        params = [named[n] for n in self._names]
        dt = _DT[self.compute_dtype]
        need_grad = torch.is_grad_enabled() and any(q.requires_grad for q in self.parameters())
        if not need_grad:
            with torch.no_grad():
                return _VitFn.forward(_Ctx(), images, self, "vit.", None, dt, self.depth, *params)
        return _VitFn.apply(images, self, "vit.", GradSink(self), dt, self.depth, *params)


class _Ctx:
    """Stand-in autograd context for inference calls (no backward)."""
