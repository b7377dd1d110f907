#!/bin/bash
# GEMM tile sweep (tiled kernel only above the streaming threshold): default, then forced configs
R=$GRAFT_REPO_ROOT; TAG=${1:-g}; CFGS=${2:-"0 1 2 3 4 5 6 7 8 9 10 11 12"}
cd $R; mkdir -p gpurun_out
{ echo "== default"; timeout -k 10 120 tools/kbench pw 256 || exit $?
  for c in $CFGS; do echo "== cfg $c"; timeout -k 10 120 tools/kbench pw 256 100000 $c || exit $?; done
} > gpurun_out/kt_$TAG.log 2>&1
echo done $?
