"""CPU restatements (plain PyTorch fp32) of the reference's hot-path modules -- ORACLE.

Test infrastructure only (see ``oracle/__init__.py``).  Each function/class cites the
reference code it restates; ``tests/test_oracle_golden.py`` pins every one of them against
fixtures produced by running the reference itself (``tests/golden/make_golden.py``).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import b0_cpu


class DetectorCPU(nn.Module):
    """``PretrainedBackboneDetector('efficientnet_b0')`` (src/pretrained_detector.py:15-143):
    trunk = timm children()[:-1] (:46), temporal attention (:65-71), head (:74-76),
    forward (:103-143).  Same state_dict keys as the reference."""

    def __init__(self, num_classes=2, dropout_rate=0.5, use_temporal_attention=True):
        super().__init__()
        self.backbone = b0_cpu.trunk(b0_cpu.EfficientNetB0())
        self.use_temporal_attention = use_temporal_attention
        if use_temporal_attention:
            self.temporal_attention = nn.Sequential(nn.Linear(1280, 64), nn.ReLU(), nn.Linear(64, 1), nn.Sigmoid())
        self.dropout = nn.Dropout(dropout_rate)
        self.fc1 = nn.Linear(1280, 256)
        self.fc2 = nn.Linear(256, num_classes)

    def forward(self, x):
        b, t, c, h, w = x.shape
        f = self.backbone(x.reshape(b * t, c, h, w)).view(b, t, -1)
        if self.use_temporal_attention:
            a = F.softmax(self.temporal_attention(f).squeeze(-1), dim=1)
            g = (f * a.unsqueeze(-1)).sum(dim=1)
        else:
            g = f.mean(dim=1)
            a = torch.ones(b, t) / t
        z = self.fc2(self.dropout(F.relu(self.fc1(self.dropout(g)))))
        return z, a


class LogicCellCPU(nn.Module):
    """``LogicCell`` (src/RNNModel.py:5-41)."""

    def __init__(self, input_size, hidden_size):
        super().__init__()
        self.hidden_size = hidden_size
        self.and_gate = nn.Linear(input_size + hidden_size, hidden_size)
        self.or_gate = nn.Linear(input_size + hidden_size, hidden_size)
        self.not_gate = nn.Linear(hidden_size, hidden_size)
        self.forget_gate = nn.Linear(input_size + hidden_size, hidden_size)
        self.input_gate = nn.Linear(input_size + hidden_size, hidden_size)
        self.cell_gate = nn.Linear(input_size + hidden_size, hidden_size)
        self.output_gate = nn.Linear(input_size + hidden_size, hidden_size)

    def forward(self, x, h, c):
        u = torch.cat((x, h), dim=1)
        a = torch.sigmoid(self.and_gate(u))
        o_ = torch.sigmoid(self.or_gate(u))
        n = torch.tanh(self.not_gate(h))
        f = torch.sigmoid(self.forget_gate(u))
        i = torch.sigmoid(self.input_gate(u))
        g = torch.tanh(self.cell_gate(u))
        c1 = f * c + i * g
        c2 = a * c1 + o_ * n
        o = torch.sigmoid(self.output_gate(u))
        return o * torch.tanh(c2), c2


class LogicRNNLSTMCPU(nn.Module):
    """``LogicRNNLSTM`` (src/RNNModel.py:43-147) incl. its quirks: batch sorted by length and
    never un-sorted (:92-95); all layers share one (h, c) per step (:103-115, F8d)."""

    def __init__(self, input_size=1024, hidden_size=512, num_layers=2, dropout=0.5):
        super().__init__()
        self.hidden_size, self.num_layers = hidden_size, num_layers
        self.logic_cells = nn.ModuleList([LogicCellCPU(input_size if i == 0 else hidden_size, hidden_size)
                                          for i in range(num_layers)])
        self.dropout = nn.Dropout(dropout)
        self.attention = nn.Sequential(nn.Linear(hidden_size, hidden_size), nn.Tanh(), nn.Linear(hidden_size, 1),
                                       nn.Softmax(dim=1))
        self.classifier = nn.Sequential(nn.Linear(hidden_size, hidden_size), nn.ReLU(), nn.Dropout(dropout),
                                        nn.Linear(hidden_size, 1))

    def forward(self, x, lengths=None):
        b, t, _ = x.shape
        if lengths is not None:
            lengths, idx = lengths.sort(0, descending=True)
            x = x[idx]
        h = torch.zeros(b, self.hidden_size)
        c = torch.zeros(b, self.hidden_size)
        outs = []
        for s in range(t):
            hh, cc = h, c
            for i, cell in enumerate(self.logic_cells):
                hh, cc = cell(x[:, s] if i == 0 else hh, hh, cc)
                if i < self.num_layers - 1:
                    hh = self.dropout(hh)
            outs.append(hh)
            h, c = hh, cc
        o = torch.stack(outs, dim=1)
        if lengths is not None:
            mask = (torch.arange(t).expand(b, t) < lengths.unsqueeze(1)).float().unsqueeze(-1)
            o = o * mask
        w = self.attention(o)
        return torch.sigmoid(self.classifier((w * o).sum(dim=1)))

    def predict(self, x, lengths=None):
        with torch.no_grad():
            return (self.forward(x, lengths) >= 0.5).float()


class CNNLSTMHybridCPU(nn.Module):
    """``CNNLSTMHybrid`` (src/models.py:20-85)."""

    def __init__(self, input_channels=3, hidden_size=256, num_layers=2, num_classes=2, dropout=0.3):
        super().__init__()
        self.cnn = nn.Sequential(
            nn.Conv2d(input_channels, 64, 7, 2, 3), nn.BatchNorm2d(64), nn.ReLU(), nn.MaxPool2d(3, 2, 1),
            nn.Conv2d(64, 128, 5, 1, 2), nn.BatchNorm2d(128), nn.ReLU(), nn.MaxPool2d(3, 2, 1),
            nn.Conv2d(128, 256, 3, 1, 1), nn.BatchNorm2d(256), nn.ReLU(), nn.MaxPool2d(3, 2, 1),
            nn.Conv2d(256, 512, 3, 1, 1), nn.BatchNorm2d(512), nn.ReLU(), nn.AdaptiveAvgPool2d(1), nn.Flatten())
        self.lstm = nn.LSTM(512, hidden_size, num_layers, dropout=dropout if num_layers > 1 else 0,
                            batch_first=True)
        self.attention = nn.Sequential(nn.Linear(hidden_size, hidden_size), nn.Tanh(), nn.Linear(hidden_size, 1))
        self.classifier = nn.Sequential(nn.Linear(hidden_size, 128), nn.ReLU(), nn.Dropout(dropout),
                                        nn.Linear(128, num_classes))

    def forward(self, x):
        b, t, c, h, w = x.shape
        f = self.cnn(x.reshape(b * t, c, h, w)).view(b, t, 512)
        o, _ = self.lstm(f)
        a = torch.softmax(self.attention(o), dim=1)
        return self.classifier((a * o).sum(dim=1))


def collate_cnn_lstm(batch, max_frames=16, image_size=(224, 224)):
    """``collate_batch_cnn_lstm`` (src/train.py:38-61): linspace-sample or last-frame-pad to 16."""
    frames, labels = [], []
    for item in batch:
        faces = item["faces"]
        m = faces.shape[0]
        if m >= max_frames:
            sel = faces[np.linspace(0, m - 1, max_frames).astype(int)]
        elif m == 0:
            sel = np.zeros((max_frames, image_size[0], image_size[1], 3), dtype=np.uint8)
        else:
            sel = np.concatenate([faces, np.repeat(faces[-1][None], max_frames - m, axis=0)], axis=0)
        frames.append(sel)
        labels.append(item["label"] if item["label"] is not None else -1)
    x = torch.from_numpy(np.stack(frames)).permute(0, 1, 4, 2, 3).float() / 255.0
    return x, torch.tensor(labels, dtype=torch.long)


def normalize_adjacency(a):
    """``normalize_adjacency`` (src/utils.py:95-104): D^-1/2 (A + I) D^-1/2 in float32."""
    a = a.astype(np.float32) + np.eye(a.shape[0], dtype=np.float32)
    d = np.power(np.sum(a, axis=1), -0.5)
    d[np.isinf(d)] = 0.0
    dm = np.diag(d)
    return dm @ a @ dm


def collate_vit_gcn(batch, max_nodes=16, image_size=(224, 224)):
    """``collate_batch`` (src/train.py:62-100): the same sampling as the CNN-LSTM collate, plus a
    chain graph over the nodes, symmetric-normalised per clip."""
    x, labels = collate_cnn_lstm(batch, max_frames=max_nodes, image_size=image_size)
    b, n = x.shape[0], x.shape[1]
    a = np.zeros((n, n), dtype=np.float32)
    for i in range(n - 1):
        a[i, i + 1] = a[i + 1, i] = 1.0
    a_norm = torch.from_numpy(np.stack([normalize_adjacency(a) for _ in range(b)])).float()
    return x, a_norm, labels


def train_step(model, x, labels, opt, class_weights=None, max_norm=1.0):
    """One step of ``EnsembleTrainer.train_epoch`` (src/ensemble_trainer.py:182-203):
    zero_grad -> forward -> weighted CE -> backward -> clip_grad_norm_(1.0) -> step."""
    opt.zero_grad()
    out = model(x)
    logits = out[0] if isinstance(out, tuple) else out
    loss = F.cross_entropy(logits, labels, weight=class_weights)
    loss.backward()
    torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=max_norm)
    opt.step()
    return float(loss)
