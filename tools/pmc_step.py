"""Per-kernel PMC table of the B0 training step from tools/pmc_step.sh's four passes.

usage: python tools/pmc_step.py gpurun_out/pmc_step_TAG [out.txt]

Per kernel (template instance), summed over every dispatch of the profiled run (1 warm-up + 2
timed steps + bench.py's extra step), per step = / 4:
  us        kernel time per step (PMC-pass timestamps: inflated by the profiler, weights only)
  valu%     SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES        (both quad-cycles)
  wait%     SQ_WAIT_ANY / SQ_WAVE_CYCLES                (waiting on memory / dependencies)
  iwait%    SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES           (waiting for an instruction's inputs)
  ldsc%     SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE    (LDS cycles lost to bank conflicts)
  mfma%     SQ_VALU_MFMA_BUSY_CYCLES / (time x 2.4 GHz x 1024 SIMDs)  (estimate)
  fetchMB / writeMB  raw FETCH_SIZE / WRITE_SIZE per step (KiB x 1024; FETCH reads 0.5x for
            contiguous 16-B/lane streams and 1.0x for 64-B channel slices -- tools/pmc_traffic.py)
"""
import collections
import csv
import glob
import os
import sys

STEPS = 4.0


def rows(d, p):
    f = glob.glob(os.path.join(d, p, "**", "*counter_collection.csv"), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def main():
    d = sys.argv[1]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    tim = collections.defaultdict(float)
    seen = set()
    for p in ("p1", "p2", "p3", "p4"):
        for r in rows(d, p):
            n = r["Kernel_Name"].split("(")[0]
            if "dfd::" not in n:
                continue
            agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
            key = (p, r["Dispatch_Id"])
            if p == "p1" and key not in seen:
                seen.add(key)
                tim[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    out = []
    hdr = f"{'us/step':>8} {'valu%':>6} {'wait%':>6} {'iwait%':>6} {'ldsc%':>6} {'mfma%':>6} {'fetchMB':>8} {'writeMB':>8}  kernel"
    out.append(hdr)
    tot_t = sum(tim.values()) / STEPS
    for n in sorted(tim, key=lambda k: -tim[k]):
        c = agg[n]
        t = tim[n] / STEPS
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        lds = c.get("SQ_LDS_IDX_ACTIVE", 0) or 1
        mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (tim[n] * 1e-6 * 2.4e9 * 1024) * 100 if tim[n] else 0
        out.append(f"{t:8.1f} {100 * c.get('SQ_ACTIVE_INST_VALU', 0) / wc:6.1f} {100 * c.get('SQ_WAIT_ANY', 0) / wc:6.1f} "
                   f"{100 * c.get('SQ_WAIT_INST_ANY', 0) / wc:6.1f} {100 * c.get('SQ_LDS_BANK_CONFLICT', 0) / lds:6.1f} "
                   f"{mf:6.1f} {c.get('FETCH_SIZE', 0) * 1024 / STEPS / 1e6:8.1f} "
                   f"{c.get('WRITE_SIZE', 0) * 1024 / STEPS / 1e6:8.1f}  {n[:100]}")
    out.append(f"total kernel time per step (profiled) {tot_t:.1f} us")
    text = "\n".join(out)
    print(text)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text + "\n")


if __name__ == "__main__":
    main()
