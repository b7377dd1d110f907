#!/bin/bash
# round-5 call J: the fused projection backward run twice per storage type (tools/pwl_det); variant
# binaries built from other compile flags of k_pwl_bwd.hip
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r05; mkdir -p $O
for b in pwl_det_noslp; do
  echo "== $b"; timeout -k 10 300 ./tools/$b > $O/j_$b.log 2>&1 || { cat $O/j_$b.log; exit 1; }
  grep "F32" $O/j_$b.log | cut -c1-200
done
