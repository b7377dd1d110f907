import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

import deepfake_amd  # noqa: E402,F401  (registers the package alias)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def have_gpu() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


@pytest.fixture(params=["default", "forced", "split_dw"])
def kernel_paths(request):
    """Run a test with the production kernel selection ("default": the streaming 1x1 kernels and the
    BN-folded conv_pw backward only on >= 100K-row layers, fused depthwise backward), with the first
    two forced onto every covered layer ("forced", so the small parity shapes exercise the
    high-resolution code paths too), and with the depthwise backward as two kernels ("split_dw")."""
    from deepfake_amd import backbone
    knobs = {"default": {}, "forced": {"stream_min_rows": 0, "fold_min_rows": 0},
             "split_dw": {"dw_bwd_fused": 0}}[request.param]
    prev = dict(backbone.DEFAULT_TUNING)  # the plans of runtimes built inside the test take these
    backbone.DEFAULT_TUNING.update(knobs)
    try:
        yield request.param
    finally:
        backbone.DEFAULT_TUNING.clear()
        backbone.DEFAULT_TUNING.update(prev)
