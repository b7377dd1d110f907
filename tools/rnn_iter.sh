#!/bin/bash
# Recurrent-model iteration: the RNN / CNN-LSTM parity tests, the C4 benches (no CPU leg), a
# kernel-trace profile of the LogicRNN step, then the whole -m gpu suite and the B0 quick bench.
R=$GRAFT_REPO_ROOT; TAG=${1:-rnn}
cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rnn.py tests/test_cnn_lstm.py -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/trnn_$TAG.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/trnn_$TAG.log | tail -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench_temporal.py --model both --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/temporal_$TAG.jsonl 2> gpurun_out/temporal_$TAG.err || { echo BENCH FAILED; tail -20 gpurun_out/temporal_$TAG.err; exit 1; }
cut -c1-200 gpurun_out/temporal_$TAG.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/tprof_${TAG}_rnn -o run -- python $R/bench_temporal.py --model rnn --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/tprof_${TAG}_rnn.log 2>&1 || { echo "PROF rnn FAILED"; exit 1; }
echo "PROF rnn ok"
[ -n "$2" ] && exec_all=1
cd $R
if [ -n "$exec_all" ]; then
  timeout -k 10 700 python -u -m pytest tests/ -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1; rc=$?
  tail -3 gpurun_out/t_$TAG.log; [ $rc -le 1 ] || exit $rc
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bq_$TAG.json 2> gpurun_out/bq_$TAG.err || { echo BENCH FAILED; tail -5 gpurun_out/bq_$TAG.err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/bq_$TAG.json
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_$TAG.log 2>&1 || { echo PROF FAILED; exit 1; }
  echo PROF b0 ok
fi
