"""Round-4 HBM traffic table from tools/r04/traffic.sh's PMC passes -> profiles/r04/traffic.json.

usage: python tools/pmc_traffic_r04.py gpurun_out/r04/traffic [profiles/r04/traffic.json]

Per kernel instance and launch site of the B0 training step (256 frames, 224^2, bf16):
  write_bytes = WRITE_SIZE (x 1024), divided by the write calibration factor of tools/fetch_calib
                (16-B/lane stores: 1.0 in round 2; re-measured here);
  fetch_bytes = when the request-size counters exist (TCC_EA0_RDREQ and _32B / _64B / _128B):
                  32 RDREQ_32B + 64 RDREQ_64B + 128 RDREQ_128B (+ 64 per request in no class),
                validated on the calibration kernels' known byte counts (contiguous 16-B/lane and
                64-B channel-slice reads) -- the method that does not depend on the access pattern
                (FETCH_SIZE's own expression, 128 TCC_BUBBLE + 64 (RDREQ - BUBBLE - 32B) + 32 32B,
                tallies the 128-B requests of 16-B/lane streaming reads at 64 B on gfx950, round 4
                calibration: 0.5 of the known bytes); otherwise FETCH_SIZE (x 1024) divided by the
                calibration factor of the access pattern.
  algorithmic_bytes = SURVEY 8(d) / DESIGN.md section 4 per-launch figures (one read of every input,
                one write of every output).
Launch sites are assigned by the fixed backward order of the plan (blocks 6.0 -> 0.0).  The file
records the git commit of the measured tree (HEAD when this aggregator runs; the call is made from a
committed tree).
"""
import csv
import glob
import json
import os
import statistics
import subprocess
import sys

F, ES = 256, 2
KNOWN = 256 * 112 * 112 * 96 * 2  # fetch_calib's tensor, bytes per dispatch

# (stage, idx, cin, cout, mid, k, s, hin) of timm efficientnet_b0 at 224^2 (plan.cpp kArch)
ARCH = [(1, 1, 3, 1, 1, 16), (0, 2, 3, 2, 6, 24), (0, 2, 5, 2, 6, 40), (0, 3, 3, 2, 6, 80), (0, 3, 5, 1, 6, 112),
        (0, 4, 5, 2, 6, 192), (0, 1, 3, 1, 6, 320)]


def blocks():
    out, cin, h = [], 32, 112
    for si, (ds, rep, k, s, e, cout) in enumerate(ARCH):
        for bi in range(rep):
            st = s if bi == 0 else 1
            ho = (h + 2 * ((st - 1 + k - 1) // 2) - k) // st + 1
            out.append(dict(name=f"{si}.{bi}", ds=ds, cin=cin, cout=cout, mid=cin * e, k=k, s=st, hin=h, hout=ho))
            cin, h = cout, ho
    return out


def sites():
    """per-step dispatch order of the three kernel classes in the backward, with algorithmic bytes"""
    bl = blocks()
    dw1, dw2, apply1 = [], [], []
    for b in reversed(bl):
        Min, Mout, C = F * b["hin"] ** 2, F * b["hout"] ** 2, b["mid"]
        # BN3 backward apply (all blocks but 0.0, whose fused projection kernel applies it in its staging)
        if b["name"] != "0.0":
            apply1.append((f"bn3 {b['name']}", 3 * ES * Mout * b["cout"]))
        if b["s"] == 1:
            dw1.append((b["name"], ES * 4 * Mout * C + 4 * b["k"] ** 2 * C))
        else:
            dw2.append((b["name"], ES * (2 * Min * C + 2 * Mout * C) + 8 * b["k"] ** 2 * C))
        # BN1 backward apply of the non-fold conv_pw blocks (Min < 100,000 rows)
        if not b["ds"] and Min < 100000:
            apply1.append((f"bn1 {b['name']}", 3 * ES * Min * C))
    return {"dw_bwd1_kernel": dw1, "dw_bwd2_kernel": dw2, "bn_bwd_apply_kernel<dfd::bf16, 1>": apply1}


def read(d, sub):
    fs = glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True)
    if not fs:
        return None
    rows = list(csv.DictReader(open(fs[0])))
    per = {}
    for r in rows:
        key = (int(r["Dispatch_Id"]), r["Kernel_Name"].split("(")[0])
        per.setdefault(key, {})[r["Counter_Name"]] = per.get(key, {}).get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [(k[1], v) for k, v in sorted(per.items())]


def raw_bytes(c):
    rd, r32 = c["TCC_EA0_RDREQ_sum"], c["TCC_EA0_RDREQ_32B_sum"]
    r64, r128 = c["TCC_EA0_RDREQ_64B_sum"], c["TCC_EA0_RDREQ_128B_sum"]
    return 32 * r32 + 64 * r64 + 128 * r128 + 64 * max(0.0, rd - r32 - r64 - r128)


def calib(d, sub, fn):
    rows = read(d, sub)
    if not rows:
        return None
    return statistics.median(fn(c) for _, c in rows) / KNOWN


def per_site(rows, cls, fn):
    """values of one kernel class, dispatch order, chunked into steps; median per site"""
    vals = [fn(c) for n, c in rows if cls in n]
    n = len(sites()[cls])
    steps = [vals[i:i + n] for i in range(0, len(vals) - n + 1, n)]
    return [statistics.median(s[j] for s in steps) for j in range(n)], len(steps)


def main():
    d = sys.argv[1]
    dst = sys.argv[2] if len(sys.argv) > 2 else "profiles/r04/traffic.json"
    cal = {f"fetch_mode{m}": calib(d, f"calib_f{m}", lambda c: c["FETCH_SIZE"] * 1024) for m in range(3)}
    cal.update({f"write_mode{m}": calib(d, f"calib_w{m}", lambda c: c["WRITE_SIZE"] * 1024) for m in (3, 4)})
    raw_ok = all(read(d, f"calib_r{m}") for m in range(3))
    if raw_ok:
        cal.update({f"raw_mode{m}": calib(d, f"calib_r{m}", raw_bytes) for m in range(3)})
        # the request-size count is exact on the contiguous pattern (mode 0); on 64-B channel slices
        # (modes 1, 2) it reads 2.0: each 64-B slice request is filled as a whole 128-B line, so it
        # counts the bytes the L2s request from the fabric at line granularity (an upper bound of the
        # HBM bytes: the other half of a line may be served by the Infinity Cache)
        raw_ok = abs(cal["raw_mode0"] - 1.0) < 0.05
    fetch, write = read(d, "fetch"), read(d, "write")
    raw = read(d, "raw") if raw_ok else None
    wf = cal["write_mode3"]
    out = {"_method": ("fetch: request-size counters 32 RDREQ_32B + 64 RDREQ_64B + 128 RDREQ_128B = the bytes "
                       "the L2s request from the fabric at line granularity (exact on tools/fetch_calib's "
                       "contiguous reads, raw_mode0; 2x the useful bytes of 64-B channel-slice reads, raw_mode1/2, "
                       "whose 64-B requests are filled as 128-B lines); fetch_size_bytes = FETCH_SIZE x 1024 "
                       "for comparison (1/2 of 128-B requests on gfx950)" if raw_ok else
                       "fetch: FETCH_SIZE / the 64-B channel-slice calibration factor (fetch_mode1)") +
                      "; write: WRITE_SIZE / write_mode3; separate rocprofv3 --pmc passes, kernel trace only",
           "_calibration": {k: (round(v, 4) if v is not None else None) for k, v in cal.items()},
           "_commit": subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], capture_output=True,
                                     text=True).stdout.strip()}
    st = sites()
    for cls, ss in st.items():
        fv, nst = per_site(raw if raw_ok else fetch, cls,
                           raw_bytes if raw_ok else (lambda c: c["FETCH_SIZE"] * 1024 / cal["fetch_mode1"]))
        fz, _ = per_site(fetch, cls, lambda c: c["FETCH_SIZE"] * 1024)
        wv, _ = per_site(write, cls, lambda c: c["WRITE_SIZE"] * 1024 / wf)
        for (site, alg), fb, fs, wb in zip(ss, fv, fz, wv):
            out[f"{cls.split('<')[0]}:{site}"] = {
                "algorithmic_bytes": alg, "fetch_bytes": round(fb), "fetch_size_bytes": round(fs),
                "write_bytes": round(wb), "hbm_bytes_per_launch": round(fb + wb),
                "traffic_over_algorithmic": round((fb + wb) / alg, 4), "steps": nst}
        tot_alg = sum(a for _, a in ss)
        tot = sum(out[f"{cls.split('<')[0]}:{s}"]["hbm_bytes_per_launch"] for s, _ in ss)
        out[f"{cls.split('<')[0]}:total"] = {"algorithmic_bytes": tot_alg, "hbm_bytes_per_step": tot,
                                             "traffic_over_algorithmic": round(tot / tot_alg, 4)}
    # the bench's probe (roofline.py reads this key)
    out["dw_bwd:1.0"] = dict(out["dw_bwd2_kernel:1.0"])
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if not k.startswith("bn_bwd_apply_kernel:b")}, indent=1))


if __name__ == "__main__":
    main()
