#!/bin/bash
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
{ echo "== default"; timeout -k 10 120 tools/kbench pw 256 || exit $?
  echo "== stream0"; timeout -k 10 120 tools/kbench pw 256 0 || exit $?
} > gpurun_out/kt_b.log 2>&1
echo done $?
