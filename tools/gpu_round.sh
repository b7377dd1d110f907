#!/bin/bash
# One GPU call: the named test files verbosely, then the whole -m gpu suite, the default bench line
# and a rocprofv3 kernel-trace/stats of the bench.  Assertion failures (rc 1) do not stop the chain;
# a crash, abort or time limit does.   usage: gpu_round.sh TAG [test files...]
R=$GRAFT_REPO_ROOT
TAG=${1:-x}; shift
cd $R
mkdir -p gpurun_out
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
if [ $# -gt 0 ]; then
  timeout -k 10 500 python -u -m pytest "$@" -v -s -m gpu --timeout 240 --timeout-method thread > gpurun_out/tnew_$TAG.log 2>&1; rc=$?
  echo "new tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|Error" gpurun_out/tnew_$TAG.log | tail -60
  ok $rc || exit $rc
fi
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1; rc=$?
echo "all gpu tests rc=$rc"; tail -4 gpurun_out/t_$TAG.log
ok $rc || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_$TAG.log 2>&1 || { echo PROF FAILED; exit 1; }
echo PROF ok
