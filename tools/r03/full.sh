#!/bin/bash
# Full round check: every -m gpu test, the default bench line (with CPU baseline and pointwise
# sweep), a rocprofv3 kernel trace of the bench, and the temporal/serving configs.
R=$GRAFT_REPO_ROOT; TAG=${1:-full}; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/tf_$TAG.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 gpurun_out/tf_$TAG.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bf_$TAG.json 2> gpurun_out/bf_$TAG.err || { echo BENCH FAILED; tail -5 gpurun_out/bf_$TAG.err; exit 1; }
cut -c1-400 gpurun_out/bf_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pf_$TAG -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pw-sweep > $R/gpurun_out/pf_$TAG.log 2>&1 || { echo PROF FAILED; exit 1; }
echo prof ok
cd $R
timeout -k 10 600 python bench_temporal.py --model all --no-cpu-baseline > gpurun_out/temporal_$TAG.jsonl 2> gpurun_out/temporal_$TAG.err || { echo TEMPORAL FAILED; tail -5 gpurun_out/temporal_$TAG.err; exit 1; }
cut -c1-300 gpurun_out/temporal_$TAG.jsonl
