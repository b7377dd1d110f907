#!/bin/bash
# GEMM tile sweep on the pointwise shapes: default dispatch, then each forced tile config (tiled GEMM only)
R=$GRAFT_REPO_ROOT; TAG=${1:-g}; CFGS=${2:-"0 1 2 3 4 5 6 7"}
cd $R; mkdir -p gpurun_out
{ echo "== default"; timeout -k 10 120 tools/kbench pw 256 || exit $?
  for c in $CFGS; do echo "== cfg $c"; timeout -k 10 120 tools/kbench pw 256 stream_min_rows=1000000000000 gemm_tile=$c || exit $?; done
} > gpurun_out/kg_$TAG.log 2>&1
echo done
