"""Turn the PMC passes of tools/pmc_calib.sh into profiles/traffic.json (read by bench.py).

Calibration (tools/fetch_calib.hip, every byte of a 616.6 MB NHWC bf16 [256*112*112][96] tensor
read or written once per dispatch; the tensor exceeds the 256 MiB Infinity Cache):

  mode 0  contiguous 16 B/lane read      -> FETCH_SIZE = 0.5 x bytes  (MI355X_MICROARCH.md §HBM)
  mode 1  64-B channel slices, 16 B/lane -> FETCH_SIZE = 1.0 x bytes
  mode 2  64-B channel slices,  8 B/lane -> FETCH_SIZE = 1.0 x bytes
  mode 3/4  slice / contiguous writes    -> WRITE_SIZE = 1.0 x bytes

The probed launch (dw_bwd2<bf16,3,8,56,14,1> of blocks.1.0, C = 96, k_dw_bwd2.hip) reads 64-B slices
of 32 channels (one channel group per workgroup, pixels 192 B apart: 16 B/lane staging loads of dZ
and y2, 4 B/lane strip loads of y1), i.e. the mode-1/2 pattern (factor 1.0 for both), so its
FETCH_SIZE is divided by the mode-1 factor.  (Layers with C = 32 -- blocks.0.0 -- read adjacent
64-B slices that merge into 128-B requests and count like mode 0: that is the round-1
"279 MB fetched vs 411 MB algorithmic" reading of dw_bwd<16,16,3,1>.)

usage: python tools/pmc_traffic.py gpurun_out/pmc_calib [profiles/traffic.json]
"""
import csv
import glob
import json
import os
import statistics
import sys

PROBE = ("dw_bwd:1.0", "dw_bwd2_kernel<dfd::bf16, 3, 8, 56, 14, 1>", 1)  # key, kernel name, calibration mode
KNOWN = 256 * 112 * 112 * 96 * 2


def _csv(d):
    return glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]


def values(d, counter, name_sub):
    out = []
    for r in csv.DictReader(open(_csv(d))):
        if name_sub in r["Kernel_Name"] and r["Counter_Name"] == counter:
            out.append(float(r["Counter_Value"]) * 1024)
    return out


def factor(d, mode, counter, kernel):
    v = values(os.path.join(d, f"calib_{mode}"), counter, kernel)
    return statistics.median(v) / KNOWN


def main():
    d = sys.argv[1]
    dst = sys.argv[2] if len(sys.argv) > 2 else "profiles/traffic.json"
    key, name, mode = PROBE
    calib = {"fetch_contig16": factor(d, 0, "FETCH_SIZE", "k_contig"),
             "fetch_slice64_16B": factor(d, 1, "FETCH_SIZE", "k_slice16"),
             "fetch_slice64_8B": factor(d, 2, "FETCH_SIZE", "k_slice8"),
             "write_slice64": factor(d, 3, "WRITE_SIZE", "k_wslice16"),
             "write_contig16": factor(d, 4, "WRITE_SIZE", "k_wcontig")}
    fe = values(os.path.join(d, "fetch"), "FETCH_SIZE", name)
    wr = values(os.path.join(d, "write"), "WRITE_SIZE", name)
    fetch = statistics.median(fe) / calib["fetch_slice64_16B"]
    write = statistics.median(wr) / calib["write_slice64"]
    alg = 2 * (2 * 256 * 112 * 112 * 96 + 2 * 256 * 56 * 56 * 96) + 8 * 9 * 96
    ent = {"hbm_bytes_per_launch": round(fetch + write), "fetch_bytes": round(fetch), "write_bytes": round(write),
           "fetch_size_raw_bytes": statistics.median(fe), "write_size_raw_bytes": statistics.median(wr),
           "calibration": {k: round(v, 4) for k, v in calib.items()},
           "dispatches": [len(fe), len(wr)], "algorithmic_bytes": alg,
           "traffic_over_algorithmic": round((fetch + write) / alg, 4),
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, one counter per pass, kernel trace only; FETCH divided "
                     "by the measured factor of the same 64-B channel-slice read pattern (tools/fetch_calib.hip)"}
    db = json.load(open(dst)) if os.path.exists(dst) else {}
    db[key] = ent
    json.dump(db, open(dst, "w"), indent=1)
    print(json.dumps(ent, indent=1))


if __name__ == "__main__":
    main()
