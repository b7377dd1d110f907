#!/bin/bash
# Round-3 GPU check: named test files (verbose), then a bench line and a rocprofv3 kernel trace.
# usage: r03_check.sh TAG [test files / node ids...]
R=$GRAFT_REPO_ROOT; TAG=${1:-x}; shift
cd $R; mkdir -p gpurun_out
if [ $# -gt 0 ]; then
  timeout -k 10 700 python -u -m pytest "$@" -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/t3_$TAG.log 2>&1; rc=$?
  echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|Error|per-layer|per-stage|256 frames" gpurun_out/t3_$TAG.log | cut -c1-2000 | tail -40
  [ $rc -le 1 ] || exit $rc
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pw-sweep > gpurun_out/b3_$TAG.json 2> gpurun_out/b3_$TAG.err || { echo BENCH FAILED; tail -5 gpurun_out/b3_$TAG.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/b3_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof3_$TAG -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pw-sweep > $R/gpurun_out/prof3_$TAG.log 2>&1 || { echo PROF FAILED; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $R/gpurun_out/prof3_$TAG.log
