"""deepfake_amd -- MI355X-native EfficientNet-B0 frame-classifier hot path.

Drop-in counterparts of the reference's hot-path API (SaiPranav1506/DeepFake-Video-Detection):

* ``PretrainedBackboneDetector`` / ``EnsembleDetector``  (src/pretrained_detector.py)
* ``EfficientNetB0Trunk`` / ``B0FrameExtractor``         (the timm trunk, src/pretrained_detector.py:43-46)
* ``WeightedCrossEntropyLoss``                           (nn.CrossEntropyLoss(weight), ensemble_trainer.py:358)
* ``FusedAdamW`` / ``FusedAdam`` / ``clip_grad_norm_``     (ensemble_trainer.py:146,199-200; train.py:323)
* ``train_step`` / ``DataParallelTrainer``                 (EnsembleTrainer.train_epoch step, ensemble_trainer.py:182-200)
* ``LogicRNNLSTM`` / ``LogicCell`` / ``create_model``       (src/RNNModel.py)
* ``CNNLSTMHybrid``                                       (src/models.py:20-85)
* ``DeepfakeModel`` / ``ViTFeatureExtractor`` / ``SimpleGCN`` (src/models.py:88-107, 199-291)

Compute runs in hand-written HIP kernels for gfx950 behind the C ABI of ``include/dfd_hip.h``
(``libdfd_hip.so``); PyTorch supplies device memory, streams and torch.distributed (RCCL).
Submodules import lazily so ``import deepfake_amd`` works before the library is built.
"""

__all__ = [
    "PretrainedBackboneDetector", "EnsembleDetector", "EfficientNetB0Trunk", "B0FrameExtractor",
    "WeightedCrossEntropyLoss", "FusedAdamW", "FusedAdam", "clip_grad_norm_", "LogicRNNLSTM", "LogicCell",
    "create_model", "CNNLSTMHybrid", "DeepfakeModel", "ViTFeatureExtractor", "SimpleGCN",
]


def __getattr__(name):
    if name in ("PretrainedBackboneDetector", "EnsembleDetector"):
        from . import pretrained_detector as m
    elif name in ("EfficientNetB0Trunk", "B0FrameExtractor"):
        from . import backbone as m
    elif name == "WeightedCrossEntropyLoss":
        from . import losses as m
    elif name in ("FusedAdamW", "FusedAdam", "clip_grad_norm_"):
        from . import optim as m
    elif name in ("LogicRNNLSTM", "LogicCell", "create_model"):
        from . import rnn as m
    elif name == "CNNLSTMHybrid":
        from . import cnn_lstm as m
    elif name in ("DeepfakeModel", "ViTFeatureExtractor", "SimpleGCN"):
        from . import vit_gcn as m
    else:
        raise AttributeError(name)
    return getattr(m, name)
