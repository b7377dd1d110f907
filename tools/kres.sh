#!/bin/bash
# Per-kernel VGPR / spill / occupancy summary of one HIP source (gfx950), e.g. tools/kres.sh k_pw_stream.hip
cd "$(dirname "$0")/../deepfake-video-detection_amd/csrc"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -c "$1" -o /tmp/kres.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | sed 's/.*remark: //' | awk '
  /Function Name:/ {name=$3}
  /VGPRs:/ && !/Spill/ {v=$2}
  /AGPRs:/ {a=$2}
  /VGPRs Spill:/ {sp=$3}
  /Occupancy/ {occ=$4}
  /LDS Size/ {printf "%-90s vgpr %4s agpr %3s spill %4s occ %s\n", substr(name,1,90), v, a, sp, occ}'
