#!/bin/bash
# Round-end evidence: full -m gpu suite, smoke(), then tools/r03/full.sh's bench / profile / temporal steps.
R=$GRAFT_REPO_ROOT; TAG=${1:-final}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1 || { echo SMOKE FAILED; tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
bash tools/r03/full.sh $TAG
