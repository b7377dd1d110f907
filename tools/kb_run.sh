#!/bin/bash
# kbench on the box: tools/kb_run.sh TAG BINARY FILTER [frames]
R=$GRAFT_REPO_ROOT; TAG=$1; B=$2; F=$3; N=${4:-256}
cd $R; mkdir -p gpurun_out
timeout -k 10 200 tools/$B "$F" $N > gpurun_out/kb_$TAG.log 2>&1; rc=$?
cat gpurun_out/kb_$TAG.log; exit $rc
