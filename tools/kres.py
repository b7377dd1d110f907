"""Print per-kernel VGPR / scratch / occupancy from hipcc -Rpass-analysis=kernel-resource-usage.

usage: python tools/kres.py deepfake-video-detection_amd/csrc/k_dw_fwd.hip [filter]
"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-c", src, "-o",
                      "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True,
                     cwd=None).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark: (.*)", line)
    if not m:
        continue
    r = m.group(1)
    if r.startswith("Function Name:"):
        cur = r.split(":", 1)[1].strip()
        rows[cur] = {}
    elif cur and ":" in r:
        k, v = r.split(":", 1)
        rows[cur][k.strip()] = v.strip().split()[0]
names = subprocess.run(["c++filt"], input="\n".join(rows), capture_output=True, text=True).stdout.splitlines()
for (mangled, d), nm in zip(rows.items(), names):
    nm = re.sub(r"\(.*", "", nm).replace("dfd::", "")
    if flt in nm:
        print("%-60s vgpr %4s agpr %4s scratch %5s occ %2s lds %6s" % (nm[:60], d.get("VGPRs"), d.get("AGPRs"),
              d.get("ScratchSize [bytes/lane]"), d.get("Occupancy [waves/SIMD]"), d.get("LDS Size [bytes/block]")))
