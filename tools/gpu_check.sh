#!/bin/bash
# parity tests, then bench, then a kernel-trace profile (each step time-limited; stops at first failure)
R=$GRAFT_REPO_ROOT
TAG=${1:-x}
cd $R
timeout -k 10 600 python -m pytest tests/ -q -x -m gpu > gpurun_out/t_$TAG.log 2>&1; rc=$?
tail -4 gpurun_out/t_$TAG.log
[ $rc -ne 0 ] && { echo "TESTS FAILED rc=$rc"; grep -E "Error|assert" gpurun_out/t_$TAG.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_$TAG.log 2>&1
echo PROF $?
