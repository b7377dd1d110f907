#!/bin/bash
# kbench A/B/C.. of several binaries on one filter, two interleaved rounds:
# tools/kb_multi.sh TAG FILTER BIN...
R=$GRAFT_REPO_ROOT; TAG=$1; F=$2; shift 2
cd $R; mkdir -p gpurun_out
for round in 1 2; do
  for b in "$@"; do
    echo "== $b (round $round)"
    timeout -k 10 120 tools/$b "$F" 256 || exit $?
  done
done > gpurun_out/kmulti_$TAG.log 2>&1
echo done
