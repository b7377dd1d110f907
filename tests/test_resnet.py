"""ResNet-50 ensemble member: ``PretrainedBackboneDetector('resnet50')`` and
``EnsembleDetector(['efficientnet_b0', 'resnet50'])`` (src/pretrained_detector.py:37-40, 146-218;
the app's default ENSEMBLE_BACKBONES, app.py:661,1597), inference.

CPU: torchvision's key names / shapes / parameter count through the oracle restatement
(oracle/resnet_cpu.py; parity against torchvision itself is unpinned: not importable here), and
the detector's state_dict layout.  GPU: eval features and logits against the fp32 oracle (rtol 1e-3,
atol 1e-5 in fp32 mode; a bf16 bound), the uint8 frame feed bit-identical to the normalised fp32
feed, the ensemble against the oracle ensemble (training: tests/test_resnet_train_gpu.py)."""
import numpy as np
import pytest
import torch

import deepfake_amd  # noqa: F401
from deepfake_amd.pretrained_detector import EnsembleDetector, PretrainedBackboneDetector
from deepfake_amd.resnet import ResNet50Trunk
from oracle.resnet_cpu import ResNet50TrunkCPU, resnet_features

IMNET = (torch.tensor([0.485, 0.456, 0.406]), torch.tensor([0.229, 0.224, 0.225]))


def _randomize_bn_(m: torch.nn.Module, seed: int) -> None:
    """Non-trivial eval statistics, so the BatchNorm folding is exercised."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                c = mod.num_features
                mod.weight.copy_(0.5 + torch.rand(c, generator=g))
                mod.bias.copy_(0.2 * torch.randn(c, generator=g))
                mod.running_mean.copy_(0.1 * torch.randn(c, generator=g))
                mod.running_var.copy_(0.5 + torch.rand(c, generator=g))


def test_trunk_keys_shapes_and_count_match_torchvision_layout():
    ours, ref = ResNet50Trunk(), ResNet50TrunkCPU()
    a, b = ours.state_dict(), ref.state_dict()
    assert list(a) == list(b)
    assert all(a[k].shape == b[k].shape for k in a)
    assert sum(p.numel() for p in ref.parameters()) == 23_508_032
    assert "4.0.downsample.0.weight" in a and "7.2.bn3.running_var" in a and "0.weight" in a


def test_detector_state_dict_and_unfreeze():
    det = PretrainedBackboneDetector("resnet50", pretrained=False)
    keys = list(det.state_dict())
    assert keys[0] == "backbone.0.weight" and "backbone.7.2.conv3.weight" in keys
    assert det.feature_dim == 2048 and tuple(det.fc1.weight.shape) == (256, 2048)
    assert "temporal_attention.0.weight" in keys and keys[-1] == "fc2.bias"
    for p in det.backbone.parameters():
        p.requires_grad = False
    det.unfreeze_backbone(2)  # reference: last two children of the trunk (layer4, avgpool)
    assert all(p.requires_grad for p in det.backbone[7].parameters())
    assert not any(p.requires_grad for p in det.backbone[6].parameters())
    with pytest.raises(RuntimeError):
        PretrainedBackboneDetector("resnet50", pretrained=True)


@pytest.mark.gpu
@pytest.mark.parametrize("size", [64, 224])
def test_features_fp32_vs_oracle(size):
    torch.manual_seed(0)
    ref = ResNet50TrunkCPU().eval()
    _randomize_bn_(ref, 1)
    ours = ResNet50Trunk("fp32")
    ours.load_state_dict(ref.state_dict())
    ours = ours.cuda().eval()
    x = torch.randn(2, 3, size, size)
    with torch.no_grad():
        want = resnet_features(ref, x)
        got = ours(x.cuda()).cpu()
    torch.testing.assert_close(got, want, rtol=1e-3, atol=1e-5)


@pytest.mark.gpu
def test_features_bf16_bound_and_uint8_feed():
    torch.manual_seed(0)
    ref = ResNet50TrunkCPU().eval()
    _randomize_bn_(ref, 2)
    rng = np.random.default_rng(0)
    u8 = torch.from_numpy(rng.integers(0, 256, (2, 224, 224, 3), dtype=np.uint8))
    xf = ((u8.float() / 255.0 - IMNET[0]) / IMNET[1]).permute(0, 3, 1, 2)
    with torch.no_grad():
        want = resnet_features(ref, xf)
    for dt in ("fp32", "bf16"):
        ours = ResNet50Trunk(dt)
        ours.load_state_dict(ref.state_dict())
        ours = ours.cuda().eval()
        with torch.no_grad():
            a = ours(xf.cuda()).cpu()
            b = ours(u8.cuda().permute(0, 3, 1, 2)).cpu()  # uint8 NHWC crops, normalised in the gather
        assert torch.equal(a, b), dt
        if dt == "fp32":
            torch.testing.assert_close(a, want, rtol=1e-3, atol=1e-5)
        else:
            rel = float((a - want).norm() / want.norm())
            assert rel < 3e-2, rel


@pytest.mark.gpu
def test_ensemble_matches_oracle():
    torch.manual_seed(0)
    ens = EnsembleDetector(["efficientnet_b0", "resnet50"], pretrained=False)
    _randomize_bn_(ens.models[1].backbone, 3)
    ens = ens.cuda().eval()
    x = torch.randn(2, 3, 3, 64, 64)
    with torch.no_grad():
        logits, scores = ens(x.cuda())
        per = [m(x.cuda()) for m in ens.models]
    torch.testing.assert_close(logits, (per[0][0] + per[1][0]) / 2)
    torch.testing.assert_close(scores, (per[0][1] + per[1][1]) / 2)
    # the resnet member against the oracle trunk + the reference head math
    m = ens.models[1]
    ref = ResNet50TrunkCPU().eval()
    ref.load_state_dict(m.backbone.state_dict())
    with torch.no_grad():
        f = resnet_features(ref, x.reshape(6, 3, 64, 64)).view(2, 3, -1)
        cpu = {k: v.detach().cpu() for k, v in m.state_dict().items()}
        h = torch.relu(f @ cpu["temporal_attention.0.weight"].T + cpu["temporal_attention.0.bias"])
        a = torch.sigmoid(h @ cpu["temporal_attention.2.weight"].T + cpu["temporal_attention.2.bias"]).squeeze(-1)
        a = torch.softmax(a, dim=1)
        g = (f * a.unsqueeze(-1)).sum(1)
        z = torch.relu(g @ cpu["fc1.weight"].T + cpu["fc1.bias"]) @ cpu["fc2.weight"].T + cpu["fc2.bias"]
    torch.testing.assert_close(per[1][0].cpu(), z, rtol=1e-3, atol=1e-5)
    torch.testing.assert_close(per[1][1].cpu(), a, rtol=1e-3, atol=1e-5)


# every distinct convolution of the ResNet-50 trunk at 224x224 (torchvision v1.5 Bottleneck):
# (Cin, H, Cout, k, stride) -- 1x1 s1 (direct A), 3x3 s1/s2 and 1x1 s2 (implicit im2col gather)
RN_CONV_SHAPES = [(64, 56, 64, 1, 1), (64, 56, 64, 3, 1), (64, 56, 256, 1, 1), (256, 56, 128, 1, 1),
                  (128, 56, 128, 3, 2), (256, 56, 512, 1, 2), (128, 28, 128, 3, 1), (512, 28, 256, 1, 1),
                  (256, 28, 256, 3, 2), (512, 28, 1024, 1, 2), (256, 14, 256, 3, 1), (1024, 14, 512, 1, 1),
                  (512, 14, 512, 3, 2), (1024, 14, 2048, 1, 2), (512, 7, 512, 3, 1), (512, 7, 2048, 1, 1)]


@pytest.mark.gpu
@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_rn_conv_kernel_every_shape(dt):
    """dfd_rn_conv (k_rnconv.hip, implicit-GEMM MFMA) against torch conv2d on the same (rounded)
    operands, with the folded-BN bias, the identity add and ReLU of the bottleneck epilogue."""
    import ctypes
    from deepfake_amd import _lib
    lib = _lib.load()
    tdt = {"fp32": torch.float32, "bf16": torch.bfloat16}[dt]
    g = torch.Generator().manual_seed(11)
    n = 3
    with torch.backends.cudnn.flags(enabled=False):
        for cin, h, cout, k, s in RN_CONV_SHAPES:
            x = torch.randn(n, h, h, cin, generator=g).to(tdt).cuda()
            w = (torch.randn(cout, k, k, cin, generator=g) / (k * k * cin) ** 0.5).to(tdt).cuda()
            b = torch.randn(cout, generator=g).cuda()
            p = (k - 1) // 2
            ho = (h + 2 * p - k) // s + 1
            res = torch.randn(n, ho, ho, cout, generator=g).to(tdt).cuda()
            out = torch.empty(n, ho, ho, cout, dtype=tdt, device="cuda")
            # (True, False): identity without ReLU -- no vgemm instantiation, the launcher's fallback
            for use_res, relu in ((False, True), (True, True), (False, False), (True, False)):
                st = _lib.stream_of(out.device)
                _lib.check(lib.dfd_rn_conv(st, 0 if dt == "fp32" else 1, x.data_ptr(), n, h, h, cin, k, k, s, p,
                                           w.data_ptr(), b.data_ptr(), res.data_ptr() if use_res else None,
                                           1 if relu else 0, cout, out.data_ptr()))
                ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2),
                                                 stride=s, padding=p).permute(0, 2, 3, 1) + b
                if dt == "bf16":
                    ref = ref.to(tdt).float()  # the epilogue rounds acc + bias before the identity add
                if use_res:
                    ref = ref + res.float()
                if relu:
                    ref = torch.relu(ref)
                got = out.float()
                if dt == "fp32":
                    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4, msg=lambda m: f"{(cin, h, cout, k, s)}: {m}")
                else:
                    rel = float((got - ref).norm() / ref.norm())
                    assert rel < 8e-3, ((cin, h, cout, k, s), use_res, relu, rel)
