"""CPU restatement (plain PyTorch fp32) of timm ``vit_base_patch16_224`` -- ORACLE.

Test infrastructure only (see ``oracle/__init__.py``).

The reference builds its ViT with ``timm.create_model('vit_base_patch16_224', pretrained=False,
num_classes=0)`` (``src/models.py:88-107``, used by ``DeepfakeModel``, ``src/models.py:222-291``,
trained by ``src/train.py:104-133``).  timm is a third-party dependency (``requirements.txt:12``,
``timm>=0.9.0``) that is neither vendored nor installed here, so this module restates timm's
published ``VisionTransformer`` for that arch string:

* ``patch_embed.proj``: Conv2d(3, 768, 16, stride 16, bias) -> flatten(2).transpose(1, 2)
* ``cls_token`` (1,1,768) prepended, ``pos_embed`` (1,197,768) added (pos_drop p=0)
* 12 x ``Block``: ``x = x + attn(norm1(x))``; ``x = x + mlp(norm2(x))`` with
  LayerNorm(768, eps=1e-6); ``attn.qkv`` Linear(768, 2304, bias) split as (3, heads=12, 64),
  softmax(q k^T * 64^-0.5) v, ``attn.proj`` Linear(768, 768); ``mlp.fc1`` Linear(768, 3072),
  exact (erf) GELU, ``mlp.fc2`` Linear(3072, 768); LayerScale / DropPath / q-k norm are identities
  at the defaults
* ``norm`` LayerNorm(768, eps=1e-6); ``global_pool='token'`` -> ``x[:, 0]``; ``fc_norm`` and
  ``head`` are identities (``num_classes=0``).

The parameter names equal timm's (``cls_token``, ``pos_embed``, ``patch_embed.proj.*``,
``blocks.{i}.{norm1,attn.qkv,attn.proj,norm2,mlp.fc1,mlp.fc2}.*``, ``norm.*``): 85,798,656
parameters.  **Parity unpinned** at the timm boundary, exactly as for the B0 trunk: no reference
test or fixture pins timm's arithmetic; the reference's own ``SimpleGCN`` / ``DeepfakeModel``
code around it is pinned by goldens generated from the reference (``tests/golden/make_golden.py``).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

EMBED, HEADS, DEPTH, MLP, PATCH, IMG = 768, 12, 12, 3072, 16, 224


class Attention(nn.Module):
    def __init__(self, dim=EMBED, heads=HEADS):
        super().__init__()
        self.heads = heads
        self.scale = (dim // heads) ** -0.5
        self.qkv = nn.Linear(dim, dim * 3, bias=True)
        self.proj = nn.Linear(dim, dim)

    def forward(self, x):
        b, n, c = x.shape
        qkv = self.qkv(x).reshape(b, n, 3, self.heads, c // self.heads).permute(2, 0, 3, 1, 4)
        q, k, v = qkv.unbind(0)
        attn = (q * self.scale) @ k.transpose(-2, -1)
        attn = attn.softmax(dim=-1)
        x = (attn @ v).transpose(1, 2).reshape(b, n, c)
        return self.proj(x)


class Mlp(nn.Module):
    def __init__(self, dim=EMBED, hidden=MLP):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.fc2 = nn.Linear(hidden, dim)

    def forward(self, x):
        return self.fc2(F.gelu(self.fc1(x)))


class Block(nn.Module):
    def __init__(self, dim=EMBED):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.attn = Attention(dim)
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = Mlp(dim)

    def forward(self, x):
        x = x + self.attn(self.norm1(x))
        return x + self.mlp(self.norm2(x))


class PatchEmbed(nn.Module):
    def __init__(self):
        super().__init__()
        self.proj = nn.Conv2d(3, EMBED, kernel_size=PATCH, stride=PATCH)

    def forward(self, x):
        return self.proj(x).flatten(2).transpose(1, 2)


class VisionTransformer(nn.Module):
    """timm ``vit_base_patch16_224`` with ``num_classes=0`` (forward -> CLS features (B, 768))."""

    def __init__(self, depth=DEPTH, img_size=IMG):
        super().__init__()
        self.num_features = EMBED
        self.patch_embed = PatchEmbed()
        n = (img_size // PATCH) ** 2
        self.cls_token = nn.Parameter(torch.zeros(1, 1, EMBED))
        self.pos_embed = nn.Parameter(torch.zeros(1, n + 1, EMBED))
        self.blocks = nn.Sequential(*[Block() for _ in range(depth)])
        self.norm = nn.LayerNorm(EMBED, eps=1e-6)

    def forward_features(self, x):
        x = self.patch_embed(x)
        x = torch.cat([self.cls_token.expand(x.shape[0], -1, -1), x], dim=1) + self.pos_embed
        return self.norm(self.blocks(x))

    def forward(self, x):
        return self.forward_features(x)[:, 0]


def create_model(name, pretrained=False, num_classes=0, **kw):
    """Stand-in for ``timm.create_model`` on the ViT arch string the reference names."""
    if name != "vit_base_patch16_224":
        raise ValueError(f"oracle ViT restates only vit_base_patch16_224, not {name!r}")
    if pretrained:
        raise RuntimeError("pretrained weights are a network fetch; unavailable offline")
    if num_classes != 0:
        raise ValueError("the reference creates the ViT with num_classes=0")
    return VisionTransformer(**kw)


class SimpleGCNCPU(nn.Module):
    """``SimpleGCN`` (src/models.py:199-219): relu(fc2(drop(relu(fc1(A_norm @ H)))))."""

    def __init__(self, in_dim, hid_dim=256, out_dim=128, dropout=0.3):
        super().__init__()
        self.fc1 = nn.Linear(in_dim, hid_dim)
        self.fc2 = nn.Linear(hid_dim, out_dim)
        self.dropout = nn.Dropout(dropout)

    def forward(self, H, A_norm):
        H = torch.bmm(A_norm, H)
        H = self.dropout(F.relu(self.fc1(H)))
        return F.relu(self.fc2(H))


class ViTFeatureExtractorCPU(nn.Module):
    """``ViTFeatureExtractor`` (src/models.py:88-107) with timm present: ``self.vit`` = the ViT."""

    def __init__(self, depth=DEPTH):
        super().__init__()
        self.vit = VisionTransformer(depth=depth)
        self.out_dim = self.vit.num_features

    def forward(self, x):
        return self.vit(x)


class DeepfakeModelCPU(nn.Module):
    """``DeepfakeModel`` (src/models.py:222-291), default ``backbone='timm_vit'`` branch:
    ViT per node -> (vit_proj = Identity at 768) -> SimpleGCN -> mean over nodes -> classifier
    Linear(128,64) / ReLU / Dropout(0.3) / Linear(64, classes).  ``depth`` < 12 only for small
    parity fixtures."""

    def __init__(self, vit_out=768, gcn_hid=256, gcn_out=128, num_classes=2, depth=DEPTH):
        super().__init__()
        self.vit = ViTFeatureExtractorCPU(depth=depth)
        self.vit_proj = nn.Identity() if vit_out == EMBED else nn.Linear(EMBED, vit_out)
        self.gcn = SimpleGCNCPU(vit_out, gcn_hid, gcn_out)
        self.classifier = nn.Sequential(nn.Linear(gcn_out, 64), nn.ReLU(), nn.Dropout(0.3),
                                        nn.Linear(64, num_classes))

    def forward(self, images, A_norm):
        b, n, c, h, w = images.shape
        feats = self.vit_proj(self.vit(images.reshape(b * n, c, h, w))).view(b, n, -1)
        g = self.gcn(feats, A_norm).mean(dim=1)
        return self.classifier(g)
