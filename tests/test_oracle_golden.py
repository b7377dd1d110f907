"""Pin the CPU oracle against golden vectors produced by running the REFERENCE itself.

The fixtures under ``tests/golden/`` were written by ``tests/golden/make_golden.py``, which
imports ``/root/reference/src`` (with ``timm``/``torchvision``/``cv2`` shims)
and records inputs, outputs, losses and gradient fingerprints.  Weights on both sides come
from the portable hash generator ``deepfake_amd.weights.deterministic_init_``.

What is pinned: the reference's head (temporal attention + fc1/fc2, ``pretrained_detector.py:
65-76,103-143``), weighted CE and the ``EnsembleTrainer.train_epoch`` step recipe
(``ensemble_trainer.py:182-200``), ``LogicRNNLSTM`` (``RNNModel.py``), ``CNNLSTMHybrid``
(``models.py:20-85``) and ``collate_batch_cnn_lstm`` (``train.py:38-61``).  The B0 trunk inside
the goldens is the oracle's own timm restatement (timm is absent): "parity unpinned" at the
timm boundary, see DESIGN.md §Parity.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn as nn

from deepfake_amd.weights import deterministic_init_, hash_uniform
from oracle import b0_cpu
from oracle.detector_cpu import (CNNLSTMHybridCPU, DetectorCPU, LogicRNNLSTMCPU, collate_cnn_lstm, collate_vit_gcn,
                                 train_step)
from b0_helpers import frames


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name))


def _check_fingerprint(named, g, prefix="g", rtol=1e-4, atol=1e-7):
    names = [str(n) for n in g[f"{prefix}_names"]]
    got = dict(named)
    assert sorted(names) == sorted(got), "parameter/tensor names differ from the reference"
    bad = []
    for i, n in enumerate(names):
        t = got[n].detach().double().flatten()
        ref_norm = float(g[f"{prefix}_norm"][i])
        if abs(float(t.norm()) - ref_norm) > rtol * ref_norm + atol:
            bad.append((n, "norm", float(t.norm()), ref_norm))
        k = min(64, t.numel())
        if not np.allclose(t[:k].numpy(), g[f"{prefix}_head"][i][:k], rtol=rtol, atol=atol):
            bad.append((n, "head"))
    assert not bad, bad[:10]


def _grads(module):
    return [(n, p.grad if p.grad is not None else torch.zeros_like(p)) for n, p in module.named_parameters()]


def test_trunk_topology_counts():
    m = b0_cpu.EfficientNetB0()
    t = b0_cpu.trunk(m)
    assert sum(p.numel() for p in t.parameters()) == 4_007_548
    bns = [mod for mod in t.modules() if isinstance(mod, nn.BatchNorm2d)]
    assert len(bns) == 49 and sum(b.num_features for b in bns) == 21_008


def test_detector_eval_golden(golden_dir):
    g = _load(golden_dir, "b0_eval_64.npz")
    det = DetectorCPU(dropout_rate=0.5)
    deterministic_init_(det, seed=int(g["seed"]))
    det.eval()
    with torch.no_grad():
        logits, scores = det(torch.from_numpy(g["x"]))
    torch.testing.assert_close(logits, torch.from_numpy(g["logits"]), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(scores, torch.from_numpy(g["frame_scores"]), rtol=1e-5, atol=1e-6)
    assert torch.allclose(scores.sum(1), torch.ones(scores.shape[0]))


def test_detector_eval_224_t1_golden(golden_dir):
    g = _load(golden_dir, "b0_eval_224_t1.npz")
    det = DetectorCPU(dropout_rate=0.5)
    deterministic_init_(det, seed=int(g["seed"]))
    det.eval()
    with torch.no_grad():
        logits, scores = det(torch.from_numpy(g["x"]))
    torch.testing.assert_close(logits, torch.from_numpy(g["logits"]), rtol=1e-5, atol=1e-6)
    assert torch.all(scores == 1.0)  # T = 1: softmax over a single frame


def test_detector_train_golden(golden_dir):
    g = _load(golden_dir, "b0_train_64.npz")
    det = DetectorCPU(dropout_rate=0.0)
    deterministic_init_(det, seed=int(g["seed"]))
    det.train()
    logits, scores = det(torch.from_numpy(g["x"]))
    crit = nn.CrossEntropyLoss(weight=torch.from_numpy(g["class_weights"]))
    loss = crit(logits, torch.from_numpy(g["labels"]))
    loss.backward()
    torch.testing.assert_close(logits.detach(), torch.from_numpy(g["logits"]), rtol=1e-5, atol=1e-6)
    assert abs(loss.item() - float(g["loss"])) <= 1e-5 * abs(float(g["loss"])) + 1e-7
    _check_fingerprint(_grads(det), g, "g")
    bufs = [(n, b) for n, b in det.named_buffers() if "running" in n]
    _check_fingerprint(bufs, g, "bn")


class _EnsembleOfOne(nn.Module):
    """``EnsembleDetector(['efficientnet_b0'], ensemble_method='average')``
    (src/pretrained_detector.py:146-218): with one member the average is the member."""

    def __init__(self):
        super().__init__()
        self.models = nn.ModuleList([DetectorCPU(dropout_rate=0.0)])

    def forward(self, x):
        logits, scores = self.models[0](x)
        return torch.stack([logits]).mean(0), torch.stack([scores]).mean(0)


def test_train_step_golden(golden_dir):
    g = _load(golden_dir, "train_step_64.npz")
    ens = _EnsembleOfOne()
    deterministic_init_(ens, seed=int(g["seed"]))
    before = {n: p.detach().clone() for n, p in ens.named_parameters()}
    opt = torch.optim.AdamW(ens.parameters(), lr=float(g["lr"]), weight_decay=float(g["wd"]))
    ens.train()
    loss = train_step(ens, torch.from_numpy(g["x"]), torch.from_numpy(g["labels"]), opt,
                      class_weights=torch.tensor([1.0, 1.0]), max_norm=1.0)
    assert abs(loss - float(g["loss"])) <= 1e-5 * abs(float(g["loss"])) + 1e-7
    deltas = [(n, p.detach() - before[n]) for n, p in ens.named_parameters()]
    _check_fingerprint(deltas, g, "delta", rtol=1e-3, atol=1e-8)


@pytest.mark.parametrize("tag", ["small", "default"])
def test_logic_rnn_golden(golden_dir, tag):
    g = _load(golden_dir, f"logic_rnn_{tag}.npz")
    m = LogicRNNLSTMCPU(int(g["input_size"]), int(g["hidden_size"]), int(g["num_layers"]), float(g["dropout"]))
    deterministic_init_(m, seed=int(g["seed"]))
    x, lengths = torch.from_numpy(g["x"]), torch.from_numpy(g["lengths"])
    m.eval()
    with torch.no_grad():
        torch.testing.assert_close(m(x, lengths), torch.from_numpy(g["y_len"]), rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(m(x), torch.from_numpy(g["y_nolen"]), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(m.predict(x, lengths), torch.from_numpy(g["pred"]))
    m.train()
    y = m(x, lengths)
    loss = torch.nn.functional.binary_cross_entropy(y, torch.from_numpy(g["target"]))
    loss.backward()
    assert abs(float(loss) - float(g["loss"])) <= 1e-5 * abs(float(g["loss"])) + 1e-7
    _check_fingerprint(_grads(m), g, "g", rtol=1e-4, atol=1e-8)


def test_logic_rnn_sort_quirk():
    """Outputs come back in length-descending order, never un-sorted (RNNModel.py:92-95, F8c)."""
    m = LogicRNNLSTMCPU(8, 6, 2, 0.0)
    deterministic_init_(m, seed=1)
    m.eval()
    x = torch.from_numpy(hash_uniform(2, "q", 3 * 5 * 8).reshape(3, 5, 8))
    lengths = torch.tensor([2, 5, 3])
    with torch.no_grad():
        y = m(x, lengths)
        ref = torch.cat([m(x[i:i + 1], lengths[i:i + 1]) for i in (1, 2, 0)])
    torch.testing.assert_close(y, ref)


def test_cnn_lstm_golden(golden_dir):
    g = _load(golden_dir, "cnn_lstm_64.npz")
    m = CNNLSTMHybridCPU(3, 256, 2, 2, 0.0)
    deterministic_init_(m, seed=int(g["seed"]))
    x = torch.from_numpy(g["x"])
    m.eval()
    with torch.no_grad():
        torch.testing.assert_close(m(x), torch.from_numpy(g["y_eval"]), rtol=1e-4, atol=1e-6)
    m.train()
    y = m(x)
    torch.testing.assert_close(y.detach(), torch.from_numpy(g["y_train"]), rtol=1e-4, atol=1e-6)
    loss = torch.nn.functional.cross_entropy(y, torch.from_numpy(g["labels"]))
    loss.backward()
    assert abs(float(loss) - float(g["loss"])) <= 1e-5 * abs(float(g["loss"])) + 1e-7
    _check_fingerprint(_grads(m), g, "g", rtol=1e-3, atol=1e-7)


def test_collate_golden(golden_dir):
    g = _load(golden_dir, "collate_cnn_lstm.npz")
    batch = []
    for i, m in enumerate(g["counts"].tolist()):
        f = (np.arange(m * 4 * 4 * 3, dtype=np.int64) * 7 + i * 13) % 256
        batch.append({"faces": f.astype(np.uint8).reshape(m, 4, 4, 3), "label": i % 2})
    x, y = collate_cnn_lstm(batch, max_frames=16, image_size=(4, 4))
    torch.testing.assert_close(x, torch.from_numpy(g["frames"]), rtol=0, atol=0)
    assert y.tolist() == g["labels"].tolist()


def test_frames_generator_matches_fixture(golden_dir):
    """The synthetic-frame generator used by the GPU tests reproduces the fixture inputs."""
    g = _load(golden_dir, "b0_eval_64.npz")
    torch.testing.assert_close(frames(1, (2, 4, 3, 64, 64)), torch.from_numpy(g["x"]), rtol=0, atol=0)


def test_collate_vit_gcn_golden(golden_dir):
    g = _load(golden_dir, "collate_vit_gcn.npz")
    batch = []
    for i, m in enumerate(g["counts"].tolist()):
        f = (np.arange(m * 4 * 4 * 3, dtype=np.int64) * 11 + i * 5) % 256
        batch.append({"faces": f.astype(np.uint8).reshape(m, 4, 4, 3), "label": i % 2})
    x, a_norm, y = collate_vit_gcn(batch, max_nodes=16, image_size=(4, 4))
    torch.testing.assert_close(x, torch.from_numpy(g["nodes"]), rtol=0, atol=0)
    torch.testing.assert_close(a_norm, torch.from_numpy(g["a_norm"]), rtol=0, atol=0)
    assert y.tolist() == g["labels"].tolist()


def test_vit_gcn_golden(golden_dir):
    """DeepfakeModel (models.py:222-291) with the ViT restatement: eval logits, train logits,
    CE loss and every gradient against the reference run (timm stand-in = oracle/vit_cpu.py)."""
    from oracle.vit_cpu import DeepfakeModelCPU
    g = _load(golden_dir, "vit_gcn_224.npz")
    m = DeepfakeModelCPU()
    deterministic_init_(m, seed=int(g["seed"]))
    x = frames(int(g["x_seed"]), tuple(int(v) for v in g["shape"]))
    a = torch.from_numpy(g["a_norm"])
    m.eval()
    with torch.no_grad():
        torch.testing.assert_close(m(x, a), torch.from_numpy(g["y_eval"]), rtol=1e-4, atol=1e-6)
    m.train()
    m.gcn.dropout.p = 0.0
    m.classifier[2].p = 0.0
    y = m(x, a)
    torch.testing.assert_close(y.detach(), torch.from_numpy(g["y_train"]), rtol=1e-4, atol=1e-6)
    loss = torch.nn.functional.cross_entropy(y, torch.from_numpy(g["labels"]))
    loss.backward()
    assert abs(float(loss) - float(g["loss"])) <= 1e-5 * abs(float(g["loss"])) + 1e-7
    _check_fingerprint(_grads(m), g, "g", rtol=1e-3, atol=1e-7)
