#!/bin/bash
# kbench A/B of compile-time variants (tools/kvariants.sh): tools/kb_var.sh TAG FILTER name1 name2 ...
# each variant runs twice, interleaved (order effects / clock drift show up as a spread)
R=$GRAFT_REPO_ROOT; TAG=${1:-v}; FILTER=$2; shift 2
cd $R; mkdir -p gpurun_out
for rep in 1 2; do
  for b in "$@"; do
    echo "== $b ($rep)"; timeout -k 10 120 tools/var/kbench_$b $FILTER 256 || exit $?
  done
done > gpurun_out/kbv_$TAG.log 2>&1
grep -E "^==|$FILTER" gpurun_out/kbv_$TAG.log
