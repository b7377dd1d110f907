#!/bin/bash
# Round evidence in one GPU call: parity tests, the default bench line, the rocprofv3
# kernel-trace/stats of the same bench command, then the PMC traffic passes.
R=$GRAFT_REPO_ROOT
TAG=${1:-r01}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -q -x -m gpu > gpurun_out/t_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/t_$TAG.log
[ $rc -ne 0 ] && { echo "TESTS FAILED rc=$rc"; exit $rc; }
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python $R/bench.py > $R/gpurun_out/prof_$TAG.log 2>&1 || { echo PROF FAILED; exit 1; }
echo PROF ok
bash $R/tools/pmc_traffic.sh
