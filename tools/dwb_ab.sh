#!/bin/bash
# A/B of compile-time kernel variants (kbench filter $KB_FILTER, default dw_bwd) (tools/kvariants.sh k_dw_bwd ...): kbench dw_bwd lines,
# every variant run twice, interleaved.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/dwb
for rep in 1 2; do
  for v in "$@"; do
    timeout -k 10 120 tools/var/kbench_$v ${KB_FILTER:-dw_bwd} > gpurun_out/dwb/${v}_$rep.txt 2>&1 || { echo "$v failed"; exit 1; }
  done
done
echo done
