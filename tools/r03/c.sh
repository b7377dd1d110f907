#!/bin/bash
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 60 tools/access_bw > gpurun_out/access_bw2.txt 2>&1 || exit $?
cat gpurun_out/access_bw2.txt
bash tools/r03/kt2.sh || exit $?
bash tools/r03/ab.sh
