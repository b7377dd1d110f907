#!/bin/bash
# kbench A/B of two binaries on one filter: tools/kb_ab.sh TAG FILTER BIN_A BIN_B [extra kbench args]
R=$GRAFT_REPO_ROOT; TAG=$1; F=$2; A=$3; B=$4; shift 4
cd $R; mkdir -p gpurun_out
{ echo "== $A"; timeout -k 10 120 tools/$A "$F" 256 "$@" || exit $?
  echo "== $B"; timeout -k 10 120 tools/$B "$F" 256 "$@" || exit $?
} > gpurun_out/kab_$TAG.log 2>&1
echo done
