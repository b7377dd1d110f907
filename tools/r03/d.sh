#!/bin/bash
# fused 7x7 MBConv + persistent recurrence: parity tests, A/Bs, kernel trace
R=$GRAFT_REPO_ROOT; TAG=${1:-d}; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v -s --timeout 200 --timeout-method thread tests/test_mbconv7_gpu.py -m gpu > gpurun_out/t_$TAG.log 2>&1; rc=$?
grep -E "PASS|FAIL|rel err|outside|Error|assert" gpurun_out/t_$TAG.log | cut -c1-600 | head -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench_temporal.py --model rnn --no-cpu-baseline > gpurun_out/rnn_$TAG.jsonl 2> gpurun_out/rnn_$TAG.err || { tail -5 gpurun_out/rnn_$TAG.err; exit 1; }
cut -c1-200 gpurun_out/rnn_$TAG.jsonl
timeout -k 10 300 python tools/ab_bench.py mbconv7 0 1 --rounds 6 --steps 5 > gpurun_out/ab_$TAG.txt 2>&1 || { tail -5 gpurun_out/ab_$TAG.txt; exit 1; }
tail -3 gpurun_out/ab_$TAG.txt
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_b0_bench_config_gpu.py tests/test_b0_224_gpu.py > gpurun_out/t2_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/t2_$TAG.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pf_$TAG -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pw-sweep > $R/gpurun_out/pf_$TAG.log 2>&1 || { echo PROF FAILED; exit 1; }
echo prof ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pfr_$TAG -o run -- python $R/bench_temporal.py --model rnn --no-cpu-baseline --steps 5 --warmup 2 > $R/gpurun_out/pfr_$TAG.log 2>&1 || { echo PROF RNN FAILED; exit 1; }
echo prof rnn ok
