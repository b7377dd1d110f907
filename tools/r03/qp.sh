#!/bin/bash
# quick check + profile: tests, bench line, rocprofv3 kernel trace
R=$GRAFT_REPO_ROOT; TAG=${1:-q}; TESTS=${2:-"tests/test_pwl_fused_gpu.py"}
cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/t_$TAG.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t_$TAG.log | head -20; exit $rc; }
bash tools/r03/prof.sh $TAG
