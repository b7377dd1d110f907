"""Turn the PMC passes of tools/pmc_traffic.sh into profiles/traffic.json (read by bench.py).

The probed launch is dw_fwd of blocks.1.0 (112x112x96 -> 56x56x96, k3 s2, bf16): kernel
dw_fwd_kernel<bf16, 8, 8, 3, 2, true, ...> on a persistent grid sized to the co-resident
workgroups; no other B0 layer uses that instance (the other stride-2 maps are not multiples of 8).  Units: FETCH_SIZE / WRITE_SIZE are KiB.  The guide (MI355X_MICROARCH.md §HBM)
documents FETCH_SIZE = RDREQ x 64 B, i.e. HALF the bytes of wide coalesced reads that issue
128-B requests.  This kernel's reads are 64-B requests -- each workgroup loads one 32-channel
bf16 slice (64 B) per pixel, the other channel groups of the pixel belong to neighbouring
workgroups -- so the raw FETCH_SIZE is taken as bytes (the input window of an 8x8 s2 tile is
17x17 pixels, a halo re-read of 17^2/16^2 = 1.13x; L2 absorbs part of it); the doubled value is
recorded next to it.  WRITE_SIZE is exact for 16-B-per-lane stores.

usage: python tools/pmc_traffic.py gpurun_out/pmc_traffic [profiles/traffic.json]
"""
import csv
import glob
import json
import os
import statistics
import sys

NAME = "dw_fwd_kernel<dfd::bf16, 8, 8, 3, 2, true"


def values(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    out = []
    for r in csv.DictReader(open(f)):
        if NAME in r["Kernel_Name"] and r["Counter_Name"] == counter:
            out.append(float(r["Counter_Value"]))
    return out


def main():
    d = sys.argv[1]
    dst = sys.argv[2] if len(sys.argv) > 2 else "profiles/traffic.json"
    fe = values(os.path.join(d, "fetch"), "FETCH_SIZE")
    wr = values(os.path.join(d, "write"), "WRITE_SIZE")
    fetch = statistics.median(fe) * 1024
    write = statistics.median(wr) * 1024
    ent = {"hbm_bytes_per_launch": round(fetch + write), "fetch_bytes": round(fetch),
           "fetch_bytes_if_128B_requests_x2": round(2 * fetch),
           "write_bytes": round(write), "fetch_size_kib_raw": statistics.median(fe),
           "write_size_kib_raw": statistics.median(wr), "dispatches": [len(fe), len(wr)],
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes, kernel trace only); "
                     "64-B read requests -> raw FETCH_SIZE taken as bytes (see tools/pmc_traffic.py)",
           "algorithmic_bytes": 2 * (256 * 112 * 112 * 96 + 256 * 56 * 56 * 96) + 4 * 9 * 96}
    db = json.load(open(dst)) if os.path.exists(dst) else {}
    db["dw_fwd:1.0"] = ent
    json.dump(db, open(dst, "w"), indent=1)
    print(json.dumps(ent))


if __name__ == "__main__":
    main()
