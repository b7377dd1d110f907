#!/bin/bash
# Build kbench binaries with compile-time variants of k_dw_bwd.hip (tools/var/kbench_<name>), for
# A/B runs of the fused depthwise backward: tools/dwb_variants.sh name "-DDWB_K5VW=2" ...
set -e
cd "$(dirname "$0")"
CSRC=../deepfake-video-detection_amd/csrc
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -fvisibility=hidden --offload-arch=gfx950 -munsafe-fp-atomics $flags \
    -c $CSRC/k_dw_bwd.hip -o var/k_dw_bwd_$name.o
  objs=$(ls $CSRC/build/*.o | grep -v '/k_dw_bwd.o$')
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -o var/kbench_$name kbench.o $objs var/k_dw_bwd_$name.o
done
