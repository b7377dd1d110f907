#!/bin/bash
# kbench A/B of the stride-1 depthwise backward variants: tools/kb_dwb1.sh TAG [binaries...]
R=$GRAFT_REPO_ROOT; TAG=${1:-k}; shift
cd $R; mkdir -p gpurun_out
for b in "$@"; do
  echo "== $b"; timeout -k 10 120 tools/$b dw_bwd 256 || exit $?
done > gpurun_out/kb_$TAG.log 2>&1
grep -E "^==|dw_bwd1|dw_bwdold" gpurun_out/kb_$TAG.log
