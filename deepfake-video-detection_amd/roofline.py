"""Roofline bookkeeping for the benchmark: algorithmic bytes/flops per launch + live kernel probe.

Algorithmic traffic follows SURVEY.md §8(d) (one read of every input, one write of every
output, weights once; BN/SiLU/SE applied in the consumers' prologues so they add no traffic):

* depthwise fwd:   es*(N*Hin*Win*C + N*Ho*Wo*C) + 4*k*k*C          (dgrad: same tensors swapped)
* depthwise wgrad: es*(N*Ho*Wo*C + N*Hin*Win*C) + 4*k*k*C
* fused depthwise backward (dgrad + wgrad + the BN2/SiLU/SE backward of its output in the staging +
  the producer's BN1/SiLU backward in the epilogue, k_dw_bwd1.hip / k_dw_bwd2.hip): reads dZ and y2
  (out map) and y1 (in map), writes dX (in map):
                   es*(2*N*Hin*Win*C + 2*N*Ho*Wo*C) + 8*k*k*C
* 1x1 fwd/dgrad:   es*(M*K + M*N) + es*N*K,  flops 2*M*N*K
* 1x1 wgrad:       es*(M*N + M*K) + 4*N*K
* SE squeeze:      es*M*C

Peaks from /opt/skills/guides/MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec; 6.29 TB/s measured
float4 copy), dense bf16 MFMA 2.5 PFLOP/s.
"""
from __future__ import annotations

import ctypes
import json
import os

from . import _lib

HBM_PEAK = 8.0e12
MFMA_BF16_PEAK = 2.5e15
KINDS = {"pw_fwd": 0, "dw_fwd": 1, "pwl_fwd": 2, "dw_dgrad": 3, "dw_wgrad": 4, "pw_dgrad": 5, "pw_wgrad": 6,
         "pwl_dgrad": 7, "pwl_wgrad": 8, "se_squeeze": 9,
         # the fused depthwise backward (k_dw_bwd.hip) is launched at the dgrad site
         "dw_bwd": 3}
_ARCH = [(1, 1, 3, 1, 1, 16), (0, 2, 3, 2, 6, 24), (0, 2, 5, 2, 6, 40), (0, 3, 3, 2, 6, 80), (0, 3, 5, 1, 6, 112),
         (0, 4, 5, 2, 6, 192), (0, 1, 3, 1, 6, 320)]


def _out(h, k, s):
    return (h + 2 * (((s - 1) + (k - 1)) // 2) - k) // s + 1


def block_geometry(H: int, W: int):
    """{(stage, idx): dict(cin, cout, mid, k, s, hin, win, hout, wout)} of the timm B0 topology."""
    h, w = _out(H, 3, 2), _out(W, 3, 2)
    cin = 32
    out = {}
    for si, (_ds, r, k, s, e, cout) in enumerate(_ARCH):
        for bi in range(r):
            st = s if bi == 0 else 1
            ho, wo = _out(h, k, st), _out(w, k, st)
            out[(si, bi)] = dict(cin=cin, cout=cout, mid=cin * e, k=k, s=st, hin=h, win=w, hout=ho, wout=wo)
            h, w, cin = ho, wo, cout
    return out


def algorithmic(kind: str, stage: int, idx: int, frames: int, H: int, W: int, es: int):
    """(bytes, flops) one launch of `kind` at block (stage, idx) moves/computes."""
    g = block_geometry(H, W)[(stage, idx)]
    Mi, Mo = frames * g["hin"] * g["win"], frames * g["hout"] * g["wout"]
    C, k = g["mid"], g["k"]
    if kind == "dw_bwd":  # reads dZ, y2 (out map) and the producer's y1 (in map), writes dX (in map); dW fp32
        return es * (2 * Mi * C + 2 * Mo * C) + 8 * k * k * C, 4 * Mo * C * k * k
    if kind in ("dw_fwd", "dw_dgrad", "dw_wgrad"):
        return es * (Mi * C + Mo * C) + 4 * k * k * C, 2 * Mo * C * k * k
    if kind == "se_squeeze":
        return es * Mo * C, Mo * C
    if kind.startswith("pwl"):
        M, K, N = Mo, g["mid"], g["cout"]
    else:
        M, K, N = Mi, g["cin"], g["mid"]
    if kind.endswith("wgrad"):
        return es * (M * N + M * K) + 4 * N * K, 2 * M * N * K
    return es * (M * K + M * N) + es * N * K, 2 * M * N * K


class KernelProbe:
    """Times one launch site of the trunk plan with HIP events during the benchmark's timed steps."""

    def __init__(self, model, kind: str, stage: int, block: int):
        self.model, self.kind, self.stage, self.block = model, kind, stage, block
        self.plan = None
        self.ms = []

    def _plan(self):
        plans = self.model.backbone.runtime().plans
        if len(plans) != 1:
            raise RuntimeError("probe expects exactly one trunk plan")
        key, h = next(iter(plans.items()))
        return key, h

    def arm(self, n: int):
        key, h = self._plan()
        self.key, self.plan = key, h
        _lib.check(_lib.load().dfd_b0_probe_arm(h, KINDS[self.kind], self.stage, self.block, n))

    def disarm(self):
        lib = _lib.load()
        buf = (ctypes.c_float * 4096)()
        cnt = ctypes.c_int()
        _lib.check(lib.dfd_b0_probe_read(self.plan, buf, 4096, ctypes.byref(cnt)))
        self.ms = [buf[i] for i in range(cnt.value)]
        _lib.check(lib.dfd_b0_probe_disarm(self.plan))

    def report(self, traffic_file: str | None = None):
        frames, H, W, dtype, _dev = self.key
        es = 2 if dtype in (1, 2) else 4  # bf16 and fp16 store 2-byte elements, fp32 4
        nbytes, flops = algorithmic(self.kind, self.stage, self.block, frames, H, W, es)
        if not self.ms:
            return None
        avg_s = sum(self.ms) / len(self.ms) / 1e3
        achieved = nbytes / avg_s / 1e9
        traffic, tsrc = None, None
        tf = traffic_file or latest_traffic_file()
        if tf and os.path.exists(tf):
            try:
                d = json.load(open(tf))
                ent = d.get(f"{self.kind}:{self.stage}.{self.block}")
                traffic = ent.get("hbm_bytes_per_launch") if ent else None
                tsrc = {"file": os.path.relpath(tf, _REPO), "commit": d.get("_commit")}
            except Exception:
                traffic = None
        return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                "frac": round(achieved / (HBM_PEAK / 1e9), 4), "traffic": traffic, "traffic_source": tsrc,
                "kernel": f"{self.kind} blocks.{self.stage}.{self.block}", "algorithmic_bytes": nbytes,
                "avg_us": round(avg_s * 1e6, 2), "launches_timed": len(self.ms)}


_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def latest_traffic_file():
    """the newest round's PMC traffic table (profiles/rNN/traffic.json, written by
    tools/pmc_traffic_r04.py from that round's rocprofv3 passes), else the round-2 profiles/traffic.json"""
    import glob

    cands = sorted(glob.glob(os.path.join(_REPO, "profiles", "r[0-9][0-9]", "traffic.json")))
    if cands:
        return cands[-1]
    old = os.path.join(_REPO, "profiles", "traffic.json")
    return old if os.path.exists(old) else None


PW_KINDS = ("pw_fwd", "pw_dgrad", "pw_wgrad", "pwl_fwd", "pwl_dgrad", "pwl_wgrad")


def pointwise_sweep(model, step, H: int, W: int, frames: int, es: int):
    """MFMA utilisation of the 1x1-conv GEMMs (north star: "MFMA utilisation on the pointwise kernels
    against the MI355X roofline"): every pointwise launch site of the 16 MBConv blocks (expansion and
    projection; forward, data and weight gradient) is timed with HIP events over one extra training
    step each, and summed: FLOPs 2*M*N*K and algorithmic bytes per launch (``algorithmic``) against
    the dense bf16 MFMA peak and the HBM peak.  The arithmetic intensity of these shapes (K, N <=
    1152) sits far below the ridge point (peak FLOP/s / peak B/s = 312 FLOP/B), so they are
    HBM-bound by construction and the MFMA fraction is reported as evidence of that, not as a target
    they can reach.  The conv_head 1x1 (320 -> 1280 at 7x7) is not a block site and is left out."""
    sites = []
    for (st, bi), g in block_geometry(H, W).items():
        for kind in PW_KINDS:
            if kind.startswith("pw_") and g["mid"] == g["cin"]:
                continue  # blocks.0.0 has no expansion conv
            sites.append((kind, st, bi))
    rows, tot_s, tot_f, tot_b = [], 0.0, 0, 0
    for kind, st, bi in sites:
        p = KernelProbe(model, kind, st, bi)
        p.arm(4)
        step()
        p.disarm()
        if not p.ms:
            continue
        t = sum(p.ms) / len(p.ms) / 1e3
        nb, fl = algorithmic(kind, st, bi, frames, H, W, es)
        rows.append({"site": f"{kind} blocks.{st}.{bi}", "us": round(t * 1e6, 2),
                     "tflops": round(fl / t / 1e12, 2), "hbm_frac": round(nb / t / HBM_PEAK, 3)})
        tot_s += t
        tot_f += fl
        tot_b += nb
    if not rows:
        return None
    best = max(rows, key=lambda r: r["tflops"])
    return {"launch_sites": len(rows), "gpu_us_per_step": round(tot_s * 1e6, 1), "flops_per_step": tot_f,
            "algorithmic_bytes_per_step": tot_b, "achieved_tflops": round(tot_f / tot_s / 1e12, 2),
            "mfma_peak_tflops": MFMA_BF16_PEAK / 1e12, "mfma_frac": round(tot_f / tot_s / MFMA_BF16_PEAK, 4),
            "hbm_frac": round(tot_b / tot_s / HBM_PEAK, 4), "arith_intensity": round(tot_f / tot_b, 1),
            "ridge_flop_per_byte": round(MFMA_BF16_PEAK / HBM_PEAK, 1), "bound": "hbm",
            "best_site": best, "sites": rows}
