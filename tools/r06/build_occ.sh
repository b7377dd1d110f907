#!/bin/bash
# Experiment (round 6): the depthwise kernels' resident-grid sizing.  Builds tools/kbench_occ<M> with the
# depthwise objects recompiled under -DDFD_OCC_PRINT (the occupancy API's answer and the kernel
# attributes on stderr) and -DDFD_OCC_MULT=<M> (grid = M x that answer).  Run on the GPU box.
# usage: build_occ.sh [f16] M...   (f16: kbench times the fp16 instantiations, tools/kbench_f16_occ<M>)
set -e
R=$(cd "$(dirname "$0")/../.." && pwd); C=$R/deepfake-video-detection_amd/csrc
HIPCC=/opt/rocm/bin/hipcc
FL="-O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable --offload-arch=gfx950 -fvisibility=hidden -munsafe-fp-atomics"
T=""
if [ "$1" = f16 ]; then T=f16; shift; fi
KB=$R/tools/kbench.o
if [ -n "$T" ]; then KB=$R/tools/kbench_f16.o; $HIPCC -O2 -std=c++17 --offload-arch=gfx950 -DKB_T=f16 -c $R/tools/kbench.hip -o $KB; fi
for M in "$@"; do
  D=$C/build_occ$M; mkdir -p $D
  for f in k_dw_bwd1 k_dw_bwd2 k_dw_fwd1 k_dw_fwd; do
    $HIPCC $FL -DDFD_OCC_PRINT -DDFD_OCC_MULT=$M -c $C/$f.hip -o $D/$f.o &
  done
  wait
  OBJS=""
  for o in $C/build/*.o; do b=$(basename $o); if [ -f $D/$b ]; then OBJS="$OBJS $D/$b"; else OBJS="$OBJS $o"; fi; done
  $HIPCC --offload-arch=gfx950 -o $R/tools/kbench${T:+_$T}_occ$M $KB $OBJS -L/opt/rocm/lib -lhipblaslt -Wl,-rpath,/opt/rocm/lib
done
