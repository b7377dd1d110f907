"""Round-6 HBM traffic table from tools/r06/traffic.sh's PMC passes -> profiles/r06/traffic.json.

usage: python tools/pmc_traffic_r06.py gpurun_out/r06/traffic [profiles/r06/traffic.json]

Same counters and calibration as tools/pmc_traffic_r04.py (request-size read count, WRITE_SIZE /
write calibration); what changed is the attribution: every pass ran with DFD_SITE_LOG, so the plan
itself logged "<class> <what> <block>" for each attributed launch in dispatch order (plan.cpp
log_site).  The i-th counter row of a kernel class is the i-th log line of that class, and the
per-site value is the median over the steps of the pass.  Algorithmic bytes per launch:
  BN-backward apply (with or without the fused finalize): read g and y, write the input gradient,
      3 * es * M * C (the stat-row reduction of the fused form adds <= 256 * 2 * C * 4 B, not counted);
  dw_bwd1: es * 4 * Mout * C + 4 k^2 C;   dw_bwd2: es * (2 Min C + 2 Mout C) + 8 k^2 C.
"""
import csv
import glob
import json
import os
import statistics
import subprocess
import sys

F, ES = 256, 2  # the bench step: 256 frames, fp16 (and bf16) storage
KNOWN = 256 * 112 * 112 * 96 * 2  # fetch_calib's tensor, bytes per dispatch
ARCH = [(1, 1, 3, 1, 1, 16), (0, 2, 3, 2, 6, 24), (0, 2, 5, 2, 6, 40), (0, 3, 3, 2, 6, 80), (0, 3, 5, 1, 6, 112),
        (0, 4, 5, 2, 6, 192), (0, 1, 3, 1, 6, 320)]
CLASSES = {"bn_bwd_apply": "bn_bwd_apply_kernel", "bn_bwd_apply_fin": "bn_bwd_apply_fin_kernel",
           "dw_bwd1": "dw_bwd1_kernel", "dw_bwd2": "dw_bwd2_kernel"}


def blocks():
    out, cin, h = {}, 32, 112
    for si, (ds, rep, k, s, e, cout) in enumerate(ARCH):
        for bi in range(rep):
            st = s if bi == 0 else 1
            ho = (h + 2 * ((st - 1 + k - 1) // 2) - k) // st + 1
            out[f"{si}.{bi}"] = dict(ds=ds, cin=cin, cout=cout, mid=cin * e, k=k, s=st, hin=h, hout=ho)
            cin, h = cout, ho
    return out


def algorithmic(cls, what, blk):
    if what == "bn_head":
        return 3 * ES * F * 7 * 7 * 1280
    b = blocks()[blk]
    Min, Mout = F * b["hin"] ** 2, F * b["hout"] ** 2
    if cls.startswith("bn_bwd_apply"):
        M, C = {"bn3": (Mout, b["cout"]), "bn2": (Mout, b["mid"]), "bn1": (Min, b["mid"])}[what]
        return 3 * ES * M * C
    if cls == "dw_bwd1":
        return ES * 4 * Mout * b["mid"] + 4 * b["k"] ** 2 * b["mid"]
    return ES * (2 * Min * b["mid"] + 2 * Mout * b["mid"]) + 8 * b["k"] ** 2 * b["mid"]


def read(d, sub):
    fs = glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True)
    if not fs:
        return None
    per = {}
    for r in csv.DictReader(open(fs[0])):
        key = (int(r["Dispatch_Id"]), r["Kernel_Name"].split("(")[0])
        per.setdefault(key, {})[r["Counter_Name"]] = per.get(key, {}).get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [(k[1], v) for k, v in sorted(per.items())]


def sites(path):
    out = {c: [] for c in CLASSES}
    for line in open(path):
        f = line.split()
        if f and f[0] in out:
            out[f[0]].append((f[1], f[2] if len(f) > 2 else ""))
    return out


def raw_bytes(c):
    rd, r32 = c["TCC_EA0_RDREQ_sum"], c["TCC_EA0_RDREQ_32B_sum"]
    r64, r128 = c["TCC_EA0_RDREQ_64B_sum"], c["TCC_EA0_RDREQ_128B_sum"]
    return 32 * r32 + 64 * r64 + 128 * r128 + 64 * max(0.0, rd - r32 - r64 - r128)


def calib(d, sub, fn):
    rows = read(d, sub)
    return statistics.median(fn(c) for _, c in rows) / KNOWN if rows else None


def attribute(rows, log, fn):
    """{(class, what, block): [per-launch values]} -- the i-th row of a class is its i-th log line"""
    out = {}
    for cls, kname in CLASSES.items():
        vals = [fn(c) for n, c in rows if n.split("<")[0].endswith(kname)]
        if len(vals) != len(log[cls]):
            raise SystemExit(f"{cls}: {len(vals)} counter rows vs {len(log[cls])} logged launches")
        for (what, blk), v in zip(log[cls], vals):
            out.setdefault((cls, what, blk), []).append(v)
    return out


def main():
    d = sys.argv[1]
    dst = sys.argv[2] if len(sys.argv) > 2 else "profiles/r06/traffic.json"
    cal = {f"fetch_mode{m}": calib(d, f"calib_f{m}", lambda c: c["FETCH_SIZE"] * 1024) for m in range(3)}
    cal.update({f"write_mode{m}": calib(d, f"calib_w{m}", lambda c: c["WRITE_SIZE"] * 1024) for m in (3, 4)})
    raw_ok = all(read(d, f"calib_r{m}") for m in range(3))
    if raw_ok:
        cal.update({f"raw_mode{m}": calib(d, f"calib_r{m}", raw_bytes) for m in range(3)})
        raw_ok = abs(cal["raw_mode0"] - 1.0) < 0.05
    wf = cal["write_mode3"]
    rsrc = ("raw", raw_bytes) if raw_ok else ("fetch", lambda c: c["FETCH_SIZE"] * 1024 / cal["fetch_mode1"])
    fv = attribute(read(d, rsrc[0]), sites(os.path.join(d, f"sites_{rsrc[0]}.txt")), rsrc[1])
    fz = attribute(read(d, "fetch"), sites(os.path.join(d, "sites_fetch.txt")), lambda c: c["FETCH_SIZE"] * 1024)
    wv = attribute(read(d, "write"), sites(os.path.join(d, "sites_write.txt")), lambda c: c["WRITE_SIZE"] * 1024 / wf)
    out = {"_method": ("fetch: request-size counters (32 RDREQ_32B + 64 RDREQ_64B + 128 RDREQ_128B: bytes the L2s "
                       "request from the fabric at line granularity)" if raw_ok else
                       "fetch: FETCH_SIZE / the 64-B channel-slice calibration factor") +
                      "; write: WRITE_SIZE / write_mode3; separate rocprofv3 --pmc passes, kernel trace only; launches "
                      "attributed by the plan's own site log (DFD_SITE_LOG), median over the pass's steps",
           "_calibration": {k: (round(v, 4) if v is not None else None) for k, v in cal.items()},
           "_commit": subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], capture_output=True,
                                     text=True).stdout.strip(),
           "_dtype": "fp16"}
    tot = {}
    for key in fv:
        cls, what, blk = key
        alg = algorithmic(cls, what, blk)
        f_, s_, w_ = statistics.median(fv[key]), statistics.median(fz[key]), statistics.median(wv[key])
        name = f"{CLASSES[cls]}:{what} {blk}".strip() if cls.startswith("bn") else f"{CLASSES[cls]}:{blk}"
        out[name] = {"algorithmic_bytes": alg, "fetch_bytes": round(f_), "fetch_size_bytes": round(s_),
                     "write_bytes": round(w_), "hbm_bytes_per_launch": round(f_ + w_),
                     "traffic_over_algorithmic": round((f_ + w_) / alg, 4), "launches": len(fv[key])}
        t = tot.setdefault(CLASSES[cls], [0, 0])
        t[0] += alg
        t[1] += f_ + w_
    for k, (a, h) in tot.items():
        out[f"{k}:total"] = {"algorithmic_bytes": a, "hbm_bytes_per_step": round(h), "traffic_over_algorithmic": round(h / a, 4)}
    out["dw_bwd:1.0"] = dict(out["dw_bwd2_kernel:1.0"])  # the bench's probe (roofline.py reads this key)
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    json.dump(out, open(dst, "w"), indent=1)
    for k, v in out.items():
        if not k.startswith("_"):
            print(f"{k:40s} alg {v['algorithmic_bytes'] / 1e6:9.2f} MB  x{v['traffic_over_algorithmic']:.3f}")


if __name__ == "__main__":
    main()
