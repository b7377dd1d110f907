"""The algorithmic byte/flop model behind bench.py's ``roofline`` field reproduces SURVEY §8(d)."""
import pytest

from deepfake_amd import roofline as R


def _totals(frames=256, H=224, es=2):
    tot = {}
    for (s, i), b in R.block_geometry(H, H).items():
        groups = [("dw%d" % b["k"], ("dw_fwd", "dw_dgrad", "dw_wgrad")), ("proj", ("pwl_fwd", "pwl_dgrad", "pwl_wgrad"))]
        if b["mid"] != b["cin"] or (s, i) != (0, 0):
            groups.append(("exp", ("pw_fwd", "pw_dgrad", "pw_wgrad")))
        for key, kinds in groups:
            for kind in kinds:
                by, fl = R.algorithmic(kind, s, i, frames, H, H, es)
                a, f = tot.get(key, (0, 0))
                tot[key] = (a + by, f + fl)
    return tot


def test_survey_totals():
    t = _totals()
    # dw3x3 20.0 GFLOP / 6.05 GB, dw5x5 33.1 / 3.32, expand 255.3 / 6.08, project 233.9 / 4.44
    assert t["dw3"][0] / 1e9 == pytest.approx(6.05, abs=0.01) and t["dw3"][1] / 1e9 == pytest.approx(20.0, abs=0.05)
    assert t["dw5"][0] / 1e9 == pytest.approx(3.32, abs=0.01) and t["dw5"][1] / 1e9 == pytest.approx(33.1, abs=0.05)
    assert t["exp"][0] / 1e9 == pytest.approx(6.08, abs=0.01) and t["exp"][1] / 1e9 == pytest.approx(255.3, abs=0.1)
    assert t["proj"][0] / 1e9 == pytest.approx(4.44, abs=0.01) and t["proj"][1] / 1e9 == pytest.approx(233.9, abs=0.1)


def test_geometry_224():
    g = R.block_geometry(224, 224)
    assert len(g) == 16
    assert g[(1, 0)] == dict(cin=16, cout=24, mid=96, k=3, s=2, hin=112, win=112, hout=56, wout=56)
    assert g[(6, 0)]["hout"] == 7 and g[(6, 0)]["cout"] == 320


def test_probe_kernel_bytes():
    # bench.py probes dw_fwd of blocks.1.0: bf16 in 112x112x96 + out 56x56x96, weights fp32
    by, fl = R.algorithmic("dw_fwd", 1, 0, 256, 224, 224, 2)
    assert by == 2 * (256 * 112 * 112 * 96 + 256 * 56 * 56 * 96) + 4 * 9 * 96
    assert fl == 2 * 256 * 56 * 56 * 96 * 9


def test_probe_fused_dw_bwd_bytes():
    # bench.py probes the fused depthwise backward of blocks.1.0 (k_dw_bwd2.hip): dZ + y2 at 56x56x96,
    # y1 read + dX written at 112x112x96 (bf16), dW fp32 read/written once
    by, fl = R.algorithmic("dw_bwd", 1, 0, 256, 224, 224, 2)
    assert by == 2 * (2 * 256 * 112 * 112 * 96 + 2 * 256 * 56 * 56 * 96) + 8 * 9 * 96
    assert fl == 4 * 256 * 56 * 56 * 96 * 9


def test_pointwise_sweep_sites_and_totals(monkeypatch):
    """The MFMA-utilisation sweep visits every 1x1 launch site once (93 = 16 blocks x 6 kinds minus
    blocks.0.0's missing expansion) and sums FLOPs / bytes / time consistently (fake probe, no GPU)."""
    armed, steps = [], []

    class FakeProbe:
        def __init__(self, model, kind, stage, block):
            self.site = (kind, stage, block)
            self.ms = []

        def arm(self, n):
            armed.append(self.site)

        def disarm(self):
            self.ms = [0.010]  # 10 us per launch

    monkeypatch.setattr(R, "KernelProbe", FakeProbe)
    out = R.pointwise_sweep(None, lambda: steps.append(1), 224, 224, 256, 2)
    assert len(armed) == len(set(armed)) == 93 == out["launch_sites"] == len(steps)
    assert all(k.startswith(("pw_", "pwl_")) for k, _, _ in armed)
    fl = sum(R.algorithmic(k, s, b, 256, 224, 224, 2)[1] for k, s, b in armed)
    assert out["flops_per_step"] == fl
    assert out["gpu_us_per_step"] == pytest.approx(930.0)
    assert out["mfma_frac"] == pytest.approx(fl / 930e-6 / R.MFMA_BF16_PEAK, rel=1e-3)
    assert out["arith_intensity"] < out["ridge_flop_per_byte"]  # HBM-bound shapes


def test_probe_report_element_size_per_dtype():
    """fp16 (plan dtype 2) stores 2-byte elements like bf16 (it was costed at 4 bytes and
    reported frac ~0.95 at the bf16 kernel's duration); fp32 4."""
    from deepfake_amd.roofline import KernelProbe, algorithmic

    for dt, es in ((0, 4), (1, 2), (2, 2)):
        p = KernelProbe(None, "dw_bwd", 1, 0)
        p.key = (256, 224, 224, dt, 0)
        p.ms = [0.4]
        r = p.report(traffic_file="/nonexistent/traffic.json")
        assert r["algorithmic_bytes"] == algorithmic("dw_bwd", 1, 0, 256, 224, 224, es)[0]
        assert abs(r["frac"] - r["algorithmic_bytes"] / 0.4e-3 / 8e12) < 1e-4
