"""Serving path and checkpoint I/O (§8(f)3) against the reference app's own outputs.

Goldens: tests/golden/make_serving_golden.py ran ``app.predict_video`` (pretrained branch,
``app.py:2027-2223``) and ``app.load_model(path, 'pretrained')`` (``app.py:1327-1769``) from a
scratch copy of the reference on the cases of tests/golden/serving_cases.py.

CPU: the result dicts of ``serving.FrameClassifierService`` for the same stub logits / env /
calibration files are EQUAL to the app's (same keys, values, descriptions; fp32 softmax on the
host as in the app); the app's tensor prep; the checkpoint loader's LAST_LOAD_STATS and refusals.
GPU: the loaded HIP detector's logits vs the app's loaded (oracle-trunk) model at the north-star
tolerance; uint8 frames normalised in the stem == normalised-first frames, bit for bit (forward
features and logits, training backward); the end-to-end service vs the CPU oracle; batched
multi-video == one video at a time; the bf16 serving bound; concurrent callers.
"""
import json
import os
import sys
import threading

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

from serving_cases import CKPT_VARIANTS, SERVE_CASES, ckpt_frames, ckpt_variant, faces_for  # noqa: E402

from deepfake_amd import checkpoint as ck  # noqa: E402
from deepfake_amd import serving  # noqa: E402

ENV_KEYS = ("MAX_FRAMES", "MIN_FACES", "DETECT_ABSTAIN_CONF", "DETECT_ABSTAIN_MARGIN", "DETECT_FAKE_THRESHOLD",
            "ALLOW_EXTREME_CALIBRATION_THRESHOLD", "FAKE_CLASS_INDEX", "DISABLE_ENHANCED_AGENT")


@pytest.fixture
def clean_env(monkeypatch):
    for k in ENV_KEYS:
        monkeypatch.delenv(k, raising=False)
    return monkeypatch


def _golden(name):
    return json.load(open(os.path.join(HERE, "golden", name)))


class StubModel(torch.nn.Module):
    def __init__(self, logits, raises=False):
        super().__init__()
        self.w = torch.nn.Parameter(torch.zeros(1))
        self.logits = torch.tensor([logits], dtype=torch.float32)
        self.raises = raises

    def forward(self, x):
        if self.raises:
            raise RuntimeError("device lost")
        t = x.shape[1]
        return self.logits.expand(x.shape[0], -1).clone(), torch.full((x.shape[0], t), 1.0 / t)


@pytest.mark.parametrize("case", SERVE_CASES, ids=[c["name"] for c in SERVE_CASES])
def test_predict_matches_reference_app(case, clean_env, tmp_path):
    gold = {r["name"]: r for r in _golden("serving_app.json")}[case["name"]]
    for k, v in case.get("env", {}).items():
        clean_env.setenv(k, v)
    ckpt = tmp_path / "checkpoint_best_efficientnet_b0.pt"
    if "calibration" in case:
        (tmp_path / "calibration_best.json").write_text(json.dumps(case["calibration"]))
    svc = serving.FrameClassifierService(StubModel(case["logits"], case.get("model_raises", False)),
                                         checkpoint_path=str(ckpt), device="cpu")
    asked = {}

    def extract(path, max_frames=16):
        asked["max_frames"] = max_frames
        return faces_for(case)

    res = svc.predict_video(str(tmp_path / "clip.mp4"), extract)
    assert asked["max_frames"] == gold["max_frames"]
    assert res == gold["result"]


def test_batch_post_processing_matches_single(clean_env):
    cases = [c for c in SERVE_CASES if not c.get("env") and not c.get("model_raises") and "calibration" not in c]
    svc = serving.FrameClassifierService(StubModel([0.3, -0.2]), device="cpu")
    faces = [faces_for(c) for c in cases]
    assert svc.predict_batch(faces) == [svc.predict_faces(f) for f in faces]


def test_tensor_prep_matches_reference_app():
    g = np.load(os.path.join(HERE, "golden", "serving_prep.npz"))
    x = torch.from_numpy(g["faces"]).permute(0, 3, 1, 2).float() / 255.0
    x = serving.imagenet_normalize(x).unsqueeze(0)
    assert torch.equal(x, torch.from_numpy(g["model_input"]))


@pytest.mark.parametrize("name", CKPT_VARIANTS)
def test_checkpoint_loader_matches_reference_app(name, tmp_path):
    gold = {r["name"]: r for r in _golden("checkpoint_load.json")["loads"]}[name]
    p = tmp_path / f"{name}_efficientnet_b0.pt"
    torch.save(ckpt_variant(name), p)
    if not gold["ok"]:
        with pytest.raises(ck.IncompatibleCheckpoint):
            ck.load_pretrained(p)
        return
    model, stats = ck.load_pretrained(p)
    assert stats == gold["stats"]
    sd = ck.normalize_state_dict_keys(ck.extract_state_dict(ckpt_variant(name)))
    msd = model.state_dict()
    for k, v in sd.items():
        if k in msd and tuple(msd[k].shape) == tuple(v.shape):
            assert torch.equal(msd[k].cpu(), v), k


@pytest.mark.parametrize("fname", ["model_resnet18.pt", "vit_base_patch16_224_best.pt"])
def test_loader_refuses_unimplemented_backbone(fname, tmp_path):
    """A checkpoint naming a backbone the MI355X path does not implement (resnet18 / ViT keyed files,
    which app.load_model would build with timm/torchvision) raises IncompatibleCheckpoint -- the
    loader's documented failure -- not the detector's ValueError."""
    p = tmp_path / fname
    torch.save({"fc1.weight": torch.zeros(256, 512), "fc1.bias": torch.zeros(256)}, p)
    with pytest.raises(ck.IncompatibleCheckpoint, match="Unsupported backbone"):
        ck.load_pretrained(p)


def test_training_checkpoint_roundtrip(tmp_path):
    """Trainer save formats (src/train.py:398-411, ensemble_trainer.py:549-571) load back through the
    app's rules with every key matched; the fused optimizer's state round-trips too."""
    from deepfake_amd.optim import FusedAdamW
    from deepfake_amd.pretrained_detector import PretrainedBackboneDetector
    from deepfake_amd.weights import deterministic_init_

    m = PretrainedBackboneDetector(pretrained=False)
    deterministic_init_(m, seed=5)
    opt = FusedAdamW(m.parameters(), lr=1e-4, weight_decay=1e-5)
    ck.save_training_checkpoint(tmp_path / "ckpt_efficientnet_b0.pt", m, optimizer=opt, epoch=2, best_f1=0.7)
    ck.save_state_dict(m, tmp_path / "best_efficientnet_b0.pt")
    for f in ("ckpt_efficientnet_b0.pt", "best_efficientnet_b0.pt"):
        m2, stats = ck.load_pretrained(tmp_path / f)
        assert stats["match_ratio"] == 1.0 and stats["missing"] == 0 and stats["unexpected"] == 0
        for (k, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
            assert torch.equal(a, b), k
    obj = torch.load(tmp_path / "ckpt_efficientnet_b0.pt", weights_only=True)
    assert set(obj) == {"epoch", "model_state", "optimizer_state", "scheduler_state", "metrics", "best_f1"}
    opt2 = FusedAdamW(PretrainedBackboneDetector(pretrained=False).parameters(), lr=1e-4)
    opt2.load_state_dict(obj["optimizer_state"])


# --------------------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("name", [n for n in CKPT_VARIANTS if n != "shape_mismatch"])
def test_loaded_detector_matches_reference_app(cuda, name, tmp_path):
    gold = {r["name"]: r for r in _golden("checkpoint_load.json")["loads"]}[name]
    if not gold["ok"]:
        pytest.skip("refused by the app (checked on CPU)")
    p = tmp_path / f"{name}_efficientnet_b0.pt"
    torch.save(ckpt_variant(name), p)
    model, _ = ck.load_pretrained(p, device=cuda)
    with torch.no_grad():
        logits, scores = model(ckpt_frames().to(cuda))
    torch.testing.assert_close(logits.cpu(), torch.tensor(gold["logits"]), rtol=1e-3, atol=1e-5)
    torch.testing.assert_close(scores.cpu(), torch.tensor(gold["frame_scores"]), rtol=1e-3, atol=1e-5)


def _faces(seed, n, size=224):
    from deepfake_amd.weights import hash_uniform

    u = hash_uniform(seed, "serving_faces", n * size * size * 3)
    return ((u + 1.0) * 127.5).astype(np.uint8).reshape(n, size, size, 3)


def _det(cuda, dtype="fp32", seed=41):
    from deepfake_amd.pretrained_detector import PretrainedBackboneDetector
    from deepfake_amd.weights import deterministic_init_

    torch.manual_seed(0)
    d = PretrainedBackboneDetector(pretrained=False, compute_dtype=dtype)
    deterministic_init_(d, seed=seed)
    return d.to(cuda)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("training", [False, True])
def test_uint8_frames_bit_identical(cuda, dtype, training):
    """Raw uint8 crops normalised in the stem == the app's prep on the host, bit for bit."""
    faces = [_faces(3 + i, 4, 96) for i in range(2)]
    u8 = torch.from_numpy(np.stack(faces)).to(cuda).permute(0, 1, 4, 2, 3)  # (B, T, 3, H, W), NHWC strides
    ref = serving.imagenet_normalize(torch.from_numpy(np.stack(faces)).permute(0, 1, 4, 2, 3).float() / 255.0)
    ref = ref.reshape(8, 3, 96, 96).contiguous(memory_format=torch.channels_last).view(2, 4, 3, 96, 96).to(cuda)
    outs = []
    for x in (u8, ref):
        det = _det(cuda, dtype).train(training)
        if training:
            det.dropout.p = 0.0
            logits, _ = det(x)
            logits.float().sum().backward()
            outs.append((logits.detach(), torch.cat([p.grad.flatten() for p in det.parameters()]),
                         det._flat_b.clone()))
        else:
            with torch.no_grad():
                logits, scores = det(x)
                feats = det.backbone(x.reshape(8, 3, 96, 96))
            outs.append((logits, scores, feats))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.gpu
def test_service_end_to_end_vs_oracle(cuda, clean_env):
    from oracle.detector_cpu import DetectorCPU
    from deepfake_amd.weights import deterministic_init_

    svc = serving.FrameClassifierService(_det(cuda).eval(), device=cuda)
    ref = DetectorCPU(dropout_rate=0.5)
    deterministic_init_(ref, seed=41)
    ref.eval()
    for i, n in enumerate((8, 3)):
        faces = _faces(20 + i, n)
        res = svc.predict_faces(faces)
        x = serving.imagenet_normalize(torch.from_numpy(faces).permute(0, 3, 1, 2).float() / 255.0).unsqueeze(0)
        with torch.no_grad():
            rl, _ = ref(x)
        exp = serving.decide(rl[0], n)
        got_logits = svc._logits([faces])
        torch.testing.assert_close(got_logits, rl, rtol=1e-3, atol=1e-5)
        assert res["prediction"] == exp["prediction"] or abs(res["prob_fake"] - exp["prob_fake"]) < 1e-4
        assert abs(res["prob_fake"] - exp["prob_fake"]) <= 1e-4
        assert set(res) == set(exp)


@pytest.mark.gpu
def test_batched_multi_video_equals_single(cuda, clean_env):
    svc = serving.FrameClassifierService(_det(cuda).eval(), device=cuda)
    vids = [_faces(30 + i, n) for i, n in enumerate((8, 8, 3, 8, 1, 3, 0))]
    batched = svc.predict_batch(vids)
    single = [svc.predict_faces(v) for v in vids]
    for b, s in zip(batched, single):
        assert set(b) == set(s)
        for k in b:
            if isinstance(b[k], float):
                assert abs(b[k] - s[k]) <= 1e-5, (k, b[k], s[k])
            else:
                assert b[k] == s[k]


@pytest.mark.gpu
def test_bf16_serving_bound(cuda, clean_env):
    """bf16 serving (opt-in) vs the fp32 oracle: |prob_fake| within 2e-2, logits within 5e-2."""
    from oracle.detector_cpu import DetectorCPU
    from deepfake_amd.weights import deterministic_init_

    svc = serving.FrameClassifierService(_det(cuda, "bf16").eval(), device=cuda)
    ref = DetectorCPU(dropout_rate=0.5)
    deterministic_init_(ref, seed=41)
    ref.eval()
    for i in range(3):
        faces = _faces(40 + i, 8)
        x = serving.imagenet_normalize(torch.from_numpy(faces).permute(0, 3, 1, 2).float() / 255.0).unsqueeze(0)
        with torch.no_grad():
            rl, _ = ref(x)
        got = svc._logits([faces])
        torch.testing.assert_close(got, rl, rtol=5e-2, atol=5e-2)
        assert abs(float(torch.softmax(got, 1)[0, 1]) - float(torch.softmax(rl, 1)[0, 1])) <= 2e-2


@pytest.mark.gpu
def test_concurrent_callers(cuda, clean_env):
    """Several threads (the app's ThreadPoolExecutor UI jobs, app.py:127-129) share one detector."""
    svc = serving.FrameClassifierService(_det(cuda).eval(), device=cuda)
    vids = [_faces(50 + i, 8 if i % 2 else 4) for i in range(8)]
    expected = [svc.predict_faces(v) for v in vids]
    got = [None] * len(vids)

    def work(i):
        with torch.cuda.stream(torch.cuda.Stream(cuda)):
            got[i] = svc.predict_faces(vids[i])

    ts = [threading.Thread(target=work, args=(i,)) for i in range(len(vids))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert got == expected
