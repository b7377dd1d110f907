"""Stage 4-6 1x1-conv backward launch sites of one median bench step (round 5):
per launch the kernel, workgroups (grid / workgroup size), VGPRs, LDS bytes and duration, in
backward order.  usage: python tools/r05/late_sites.py <rocprofv3 kernel_trace.csv>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# step boundaries: the optimizer's adam_kernel ends a step
ends = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
mid = len(ends) // 2
step = rows[ends[mid - 1] + 1:ends[mid] + 1]
# the backward starts at the first head-backward kernel; stages 4-6 are the first 9 blocks of it
start = next(i for i, r in enumerate(step) if "ce_bwd_kernel" in r["Kernel_Name"])
keys = ("pw_gemm", "pw_wgrad", "pw_sk", "pw_stream", "pwl_bwd", "dw_bwd", "reduce_slabs")
print(f"{'us':>7} {'WGs':>6} {'VGPR':>5} {'LDS':>6}  kernel")
n_dw = 0
for r in step[start:]:
    name = r["Kernel_Name"]
    if "dw_bwd" in name:
        n_dw += 1
    if n_dw > 9:  # stages 6, 5, 4: 1 + 4 + 3 blocks, and the stage-4 first block
        break
    if not any(k in name for k in keys):
        continue
    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    wgs = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]) // max(1, int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]))
    print(f"{us:7.1f} {wgs:6d} {r['VGPR_Count']:>5} {r['LDS_Block_Size']:>6}  {name[:95]}")
