"""Generate the golden fixtures under ``tests/golden/`` by running the REFERENCE code.

Runs only in the build container (it imports ``/root/reference/src``, which does
not exist on the GPU box).  The committed ``*.npz`` files are data only: inputs,
outputs, losses and gradient fingerprints; weights are regenerated from the
portable hash generator (``deepfake_amd.weights``) on both sides.

Shims: the reference imports ``torchvision`` and ``timm`` at
``src/pretrained_detector.py:9-10`` and ``cv2`` at ``src/detector.py:4``; none is
installed.  ``torchvision`` and ``cv2`` are empty stand-ins (unused on the paths
recorded here); ``timm.create_model('efficientnet_b0')`` / ``('vit_base_patch16_224')``
return the oracle's CPU restatements (``oracle/b0_cpu.py``, ``oracle/vit_cpu.py``).  The reference's own wrapping
(``children()[:-1]``), temporal attention, head, dropout/eval behaviour, loss,
clip-norm + AdamW step, ``LogicRNNLSTM``, ``CNNLSTMHybrid`` and the collate
rules are the reference's code; only the trunk arithmetic is the restatement
("parity unpinned" at the timm boundary).

Usage:  python tests/golden/make_golden.py [b0 step rnn cnn_lstm vit_gcn]
"""
from __future__ import annotations

import os
import sys
import types

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_SRC = "/root/reference/src"
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import deepfake_amd  # noqa: E402,F401
from deepfake_amd.weights import deterministic_init_, hash_uniform  # noqa: E402
from oracle import b0_cpu, vit_cpu  # noqa: E402

N_HEAD = 64  # number of leading elements of each flattened gradient stored


def _install_shims():
    tv = types.ModuleType("torchvision")
    tv.models = types.SimpleNamespace()
    tvt = types.ModuleType("torchvision.transforms")
    tv.transforms = tvt
    sys.modules.setdefault("torchvision", tv)
    sys.modules.setdefault("torchvision.transforms", tvt)
    timm = types.ModuleType("timm")

    def create_model(name, *a, **kw):
        return (vit_cpu if name.startswith("vit_") else b0_cpu).create_model(name, *a, **kw)

    timm.create_model = create_model
    sys.modules["timm"] = timm
    cv2 = types.ModuleType("cv2")
    sys.modules.setdefault("cv2", cv2)
    sys.path.insert(0, REF_SRC)


def frames(seed, shape):
    """Synthetic ImageNet-normalised frames: hash-uniform pixels in [0,1] -> app.py:1772-1780."""
    n = int(np.prod(shape))
    u = (hash_uniform(seed, "frames", n) + 1.0) * 0.5
    x = torch.from_numpy(u.reshape(shape))
    mean = torch.tensor([0.485, 0.456, 0.406]).view(1, 1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225]).view(1, 1, 3, 1, 1)
    return ((x - mean) / std).float()


def grad_fingerprint(named_params):
    names, norms, sums, heads = [], [], [], []
    for n, p in named_params:
        g = p.grad
        if g is None:
            g = torch.zeros_like(p)
        g = g.detach().double().flatten()
        names.append(n)
        norms.append(float(g.norm()))
        sums.append(float(g.sum()))
        h = np.zeros(N_HEAD)
        k = min(N_HEAD, g.numel())
        h[:k] = g[:k].numpy()
        heads.append(h)
    return dict(g_names=np.array(names), g_norm=np.array(norms), g_sum=np.array(sums), g_head=np.stack(heads))


def tensor_fingerprint(named, prefix):
    names, norms, sums, heads = [], [], [], []
    for n, t in named:
        t = t.detach().double().flatten()
        names.append(n)
        norms.append(float(t.norm()))
        sums.append(float(t.sum()))
        h = np.zeros(N_HEAD)
        k = min(N_HEAD, t.numel())
        h[:k] = t[:k].numpy()
        heads.append(h)
    return {f"{prefix}_names": np.array(names), f"{prefix}_norm": np.array(norms),
            f"{prefix}_sum": np.array(sums), f"{prefix}_head": np.stack(heads)}


def gen_b0_detector():
    import pretrained_detector as pdm

    out = {}
    # --- eval forward, B=2 clips x T=4 frames x 64x64 ---------------------------------
    torch.manual_seed(0)
    det = pdm.PretrainedBackboneDetector("efficientnet_b0", pretrained=False, num_classes=2,
                                         dropout_rate=0.5, use_temporal_attention=True)
    deterministic_init_(det, seed=0)
    det.eval()
    x = frames(1, (2, 4, 3, 64, 64))
    with torch.no_grad():
        logits, scores = det(x)
    np.savez_compressed(os.path.join(HERE, "b0_eval_64.npz"), x=x.numpy(), logits=logits.numpy(),
                        frame_scores=scores.numpy(), seed=0)
    out["b0_eval_64"] = logits

    # --- eval forward, one 224x224 frame (T=1 -> frame_scores == 1) -------
    x1 = frames(2, (1, 1, 3, 224, 224))
    with torch.no_grad():
        l1, s1 = det(x1)
    np.savez_compressed(os.path.join(HERE, "b0_eval_224_t1.npz"), x=x1.numpy(), logits=l1.numpy(),
                        frame_scores=s1.numpy(), seed=0)

    # --- train-mode forward/backward (dropout 0 for determinism), weighted CE ---------
    det = pdm.PretrainedBackboneDetector("efficientnet_b0", pretrained=False, num_classes=2,
                                         dropout_rate=0.0, use_temporal_attention=True)
    deterministic_init_(det, seed=3)
    det.train()
    x = frames(4, (3, 4, 3, 64, 64))
    labels = torch.tensor([0, 1, 1])
    cw = torch.tensor([1.5, 0.75])
    crit = torch.nn.CrossEntropyLoss(weight=cw)  # ensemble_trainer.py:358
    logits, scores = det(x)
    loss = crit(logits, labels)
    loss.backward()
    rec = dict(x=x.numpy(), labels=labels.numpy(), class_weights=cw.numpy(), logits=logits.detach().numpy(),
               frame_scores=scores.detach().numpy(), loss=np.array(float(loss)), seed=3)
    rec.update(grad_fingerprint(det.named_parameters()))
    bufs = [(n, b) for n, b in det.named_buffers() if "running" in n]
    rec.update(tensor_fingerprint(bufs, "bn"))
    np.savez_compressed(os.path.join(HERE, "b0_train_64.npz"), **rec)


def gen_train_step():
    """One EnsembleTrainer.train_epoch step (ensemble_trainer.py:158-229) on 1 batch."""
    import pretrained_detector as pdm
    from ensemble_trainer import EnsembleTrainer

    torch.manual_seed(0)
    ens = pdm.EnsembleDetector(["efficientnet_b0"], pretrained=False, num_classes=2, dropout_rate=0.0,
                               ensemble_method="average")
    deterministic_init_(ens, seed=5)
    trainer = EnsembleTrainer(ens, device="cpu", checkpoint_dir="/tmp/dfd_golden_ckpt")
    x = frames(6, (2, 3, 3, 64, 64))
    labels = torch.tensor([1, 0])
    loader = [(x, labels)]
    opt, _sched = trainer.prepare_optimizers(lr=1e-3, weight_decay=1e-5)
    cw = torch.tensor([1.0, 1.0])
    crit = torch.nn.CrossEntropyLoss(weight=cw)
    before = {n: p.detach().clone() for n, p in ens.named_parameters()}
    metrics = trainer.train_epoch(loader, opt, crit, epoch=1)
    deltas = [(n, p.detach() - before[n]) for n, p in ens.named_parameters()]
    rec = dict(x=x.numpy(), labels=labels.numpy(), loss=np.array(metrics["loss"]), lr=1e-3, wd=1e-5, seed=5)
    rec.update(tensor_fingerprint(deltas, "delta"))
    np.savez_compressed(os.path.join(HERE, "train_step_64.npz"), **rec)


def gen_logic_rnn():
    import RNNModel as R

    cfgs = {
        "small": dict(input_size=48, hidden_size=32, num_layers=2, dropout=0.0),
        "default": dict(input_size=1024, hidden_size=512, num_layers=2, dropout=0.0),
    }
    for tag, cfg in cfgs.items():
        torch.manual_seed(0)
        m = R.create_model(cfg)
        deterministic_init_(m, seed=7)
        B, T = (5, 7) if tag == "small" else (4, 16)
        x = torch.from_numpy(hash_uniform(8, "rnn_x", B * T * cfg["input_size"]).reshape(B, T, -1))
        lengths = torch.tensor([3, 7, 5, 7, 1][:B]) if tag == "small" else torch.tensor([16, 9, 16, 12])
        m.eval()
        with torch.no_grad():
            y_len = m(x, lengths)
            y_nolen = m(x)
        pred = m.predict(x, lengths)
        m.train()
        y = m(x, lengths)
        target = torch.tensor([1.0, 0.0, 1.0, 0.0, 1.0][:B]).view(B, 1)
        loss = torch.nn.functional.binary_cross_entropy(y, target)
        loss.backward()
        rec = dict(x=x.numpy(), lengths=lengths.numpy(), y_len=y_len.numpy(), y_nolen=y_nolen.numpy(),
                   pred=pred.numpy(), target=target.numpy(), loss=np.array(float(loss)), seed=7,
                   **{k: np.array(v) for k, v in cfg.items()})
        rec.update(grad_fingerprint(m.named_parameters()))
        np.savez_compressed(os.path.join(HERE, f"logic_rnn_{tag}.npz"), **rec)


def gen_cnn_lstm():
    import models as M
    import train as TR

    torch.manual_seed(0)
    m = M.CNNLSTMHybrid(3, 256, 2, 2, 0.0)
    deterministic_init_(m, seed=9)
    x = frames(10, (2, 16, 3, 64, 64))
    m.eval()
    with torch.no_grad():
        y_eval = m(x)
    m.train()
    y = m(x)
    labels = torch.tensor([1, 0])
    loss = torch.nn.functional.cross_entropy(y, labels)
    loss.backward()
    rec = dict(x=x.numpy(), y_eval=y_eval.numpy(), y_train=y.detach().numpy(), labels=labels.numpy(),
               loss=np.array(float(loss)), seed=9)
    rec.update(grad_fingerprint(m.named_parameters()))
    np.savez_compressed(os.path.join(HERE, "cnn_lstm_64.npz"), **rec)

    # collate rules (train.py:38-61) on tiny 4x4 "faces" with M = 0, 5, 16, 23 frames
    batch = []
    for i, M_ in enumerate([0, 5, 16, 23]):
        f = (np.arange(M_ * 4 * 4 * 3, dtype=np.int64) * 7 + i * 13) % 256
        batch.append({"faces": f.astype(np.uint8).reshape(M_, 4, 4, 3), "label": i % 2})
    frames_t, labels_t = TR.collate_batch_cnn_lstm(batch, max_frames=16, image_size=(4, 4))
    np.savez_compressed(os.path.join(HERE, "collate_cnn_lstm.npz"), frames=frames_t.numpy(),
                        labels=labels_t.numpy(), counts=np.array([0, 5, 16, 23]))


def gen_vit_gcn():
    """DeepfakeModel (models.py:222-291, timm ViT branch) eval + train step, and the
    vit_gcn collate rules (train.py:62-100, utils.normalize_adjacency)."""
    import models as M
    import train as TR

    # collate: tiny 4x4 faces, M = 0, 5, 16, 23 -> (B, 16, 3, 4, 4), chain-graph A_norm
    batch = []
    for i, M_ in enumerate([0, 5, 16, 23]):
        f = (np.arange(M_ * 4 * 4 * 3, dtype=np.int64) * 11 + i * 5) % 256
        batch.append({"faces": f.astype(np.uint8).reshape(M_, 4, 4, 3), "label": i % 2})
    nodes, a_norm, labels = TR.collate_batch(batch, max_nodes=16, image_size=(4, 4))
    np.savez_compressed(os.path.join(HERE, "collate_vit_gcn.npz"), nodes=nodes.numpy(), a_norm=a_norm.numpy(),
                        labels=labels.numpy(), counts=np.array([0, 5, 16, 23]))

    torch.manual_seed(0)
    m = M.DeepfakeModel()
    deterministic_init_(m, seed=12)
    B, N = 2, 3
    x = frames(13, (B, N, 3, 224, 224))
    from utils import normalize_adjacency
    A = np.zeros((N, N), dtype=np.float32)
    for i in range(N - 1):
        A[i, i + 1] = A[i + 1, i] = 1.0
    a_norm = torch.from_numpy(np.stack([normalize_adjacency(A)] * B)).float()
    m.eval()
    with torch.no_grad():
        y_eval = m(x, a_norm)
    m.train()
    m.gcn.dropout.p = 0.0
    m.classifier[2].p = 0.0
    y = m(x, a_norm)
    labels = torch.tensor([1, 0])
    loss = torch.nn.functional.cross_entropy(y, labels)
    loss.backward()
    rec = dict(x_seed=13, shape=np.array([B, N, 3, 224, 224]), a_norm=a_norm.numpy(), y_eval=y_eval.numpy(),
               y_train=y.detach().numpy(), labels=labels.numpy(), loss=np.array(float(loss)), seed=12)
    rec.update(grad_fingerprint(m.named_parameters()))
    np.savez_compressed(os.path.join(HERE, "vit_gcn_224.npz"), **rec)


def main():
    _install_shims()
    torch.set_num_threads(8)
    only = sys.argv[1:]
    for name, fn in [("b0", gen_b0_detector), ("step", gen_train_step), ("rnn", gen_logic_rnn),
                     ("cnn_lstm", gen_cnn_lstm), ("vit_gcn", gen_vit_gcn)]:
        if not only or name in only:
            fn()
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
