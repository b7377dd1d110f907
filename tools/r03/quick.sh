#!/bin/bash
# Quick check after a kernel change: selected GPU tests, kbench rows, bench line (no CPU baseline).
# usage: tools/r03/quick.sh TAG "pytest targets" "kbench filter"
R=$GRAFT_REPO_ROOT; TAG=${1:-q}; TESTS=${2:-"tests/test_b0_parity_gpu.py"}; KB=${3:-}
cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/t_$TAG.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t_$TAG.log | head -20; exit $rc; }
if [ -n "$KB" ]; then timeout -k 10 300 tools/kbench "$KB" 256 > gpurun_out/kb_$TAG.txt 2>&1 || { echo KBENCH FAILED; tail -3 gpurun_out/kb_$TAG.txt; exit 1; }; fi
timeout -k 10 600 python bench.py --no-pw-sweep --no-cpu-baseline > gpurun_out/b_$TAG.json 2> gpurun_out/b_$TAG.err || { echo BENCH FAILED; tail -5 gpurun_out/b_$TAG.err; exit 1; }
cut -c1-300 gpurun_out/b_$TAG.json
