#!/bin/bash
# C4/C5 evidence: bench_temporal.py for all three models (JSON lines), then a rocprofv3 kernel-trace
# --stats run per model.   usage: tools/temporal_round.sh TAG
R=$GRAFT_REPO_ROOT; TAG=${1:-t}
cd $R; mkdir -p gpurun_out
timeout -k 10 500 python bench_temporal.py --model all --steps 5 --warmup 2 > gpurun_out/temporal_$TAG.jsonl 2> gpurun_out/temporal_$TAG.err || { echo BENCH FAILED; tail -20 gpurun_out/temporal_$TAG.err; exit 1; }
cat gpurun_out/temporal_$TAG.jsonl
cd /tmp && export TMPDIR=/tmp
for m in rnn cnnlstm vit; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/tprof_${TAG}_$m -o run -- python $R/bench_temporal.py --model $m --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/tprof_${TAG}_$m.log 2>&1 || { echo "PROF $m FAILED"; exit 1; }
  echo "PROF $m ok"
done
