"""Per-launch duration of chosen kernels in a rocprofv3 kernel trace, in launch order within one
training step, next to the HBM floor of the matching layer (roofline.algorithmic).

usage: python tools/trace_floor.py gpurun_out/prof_v4/run_kernel_trace.csv pw_wgrad
"""
import csv
import sys
from collections import defaultdict

path, pat = sys.argv[1], sys.argv[2]
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
sel = [r for r in rows if pat in r["Kernel_Name"]]
# group by launch index within a step: the last 1/8 of launches = last step
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 8
per = len(sel) // steps
last = sel[-per:]
for r in last:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    name = r["Kernel_Name"].split("(")[0].replace("void dfd::", "")
    print("%8.1f us  grid %7s x %s  vgpr %s lds %s  %s" % (d, r["Grid_Size_X"], r["Grid_Size_Y"], r["VGPR_Count"],
                                                          r["LDS_Block_Size"], name))
