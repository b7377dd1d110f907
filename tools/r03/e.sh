#!/bin/bash
# fused 7x7 phase timing (kbench mb7) + per-cell recurrent launches: tests, bench, trace
R=$GRAFT_REPO_ROOT; TAG=${1:-e}; cd $R; mkdir -p gpurun_out
# kbench rnn: tools/kbench rnn
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_rnn.py tests/test_sgemm_gpu.py -m gpu > gpurun_out/t_$TAG.log 2>&1; rc=$?
grep -E "FAIL|Error|assert|passed|failed" gpurun_out/t_$TAG.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench_temporal.py --model rnn --no-cpu-baseline > gpurun_out/rnn_$TAG.jsonl 2> gpurun_out/rnn_$TAG.err || { tail -5 gpurun_out/rnn_$TAG.err; exit 1; }
cut -c1-160 gpurun_out/rnn_$TAG.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pfr_$TAG -o run -- python $R/bench_temporal.py --model rnn --no-cpu-baseline --steps 5 --warmup 2 > $R/gpurun_out/pfr_$TAG.log 2>&1 || { echo PROF RNN FAILED; exit 1; }
echo prof rnn ok
