#!/bin/bash
# quick A/B: the parity tests that cover the changed kernels, a plain bench, then bench + kernel stats
R=$GRAFT_REPO_ROOT; TAG=${1:-q}; shift
cd $R; mkdir -p gpurun_out
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u -m pytest "$@" -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/tq_$TAG.log 2>&1; rc=$?
  tail -2 gpurun_out/tq_$TAG.log; [ $rc -le 1 ] || exit $rc
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bq_$TAG.json 2> gpurun_out/bq_$TAG.err || { echo BENCH FAILED; tail -5 gpurun_out/bq_$TAG.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bq_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_$TAG.log 2>&1 || { echo PROF FAILED; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $R/gpurun_out/prof_$TAG.log
