#!/bin/bash
# Round-5 evidence on the current tree: smoke, every -m gpu test, the default bench line (CPU baseline
# + pointwise sweep), a rocprofv3 kernel trace of the bench, the temporal / serving lines.
R=$GRAFT_REPO_ROOT; TAG=${1:-full}; cd $R; O=gpurun_out/r05; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_$TAG.log 2>&1 || { echo SMOKE FAILED; tail -5 $O/smoke_$TAG.log; exit 1; }
tail -1 $O/smoke_$TAG.log
timeout -k 10 1000 python -u -m pytest tests/ -q -m gpu --timeout 300 --timeout-method thread > $O/tf_$TAG.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 $O/tf_$TAG.log; grep -E "^FAILED" $O/tf_$TAG.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bf_$TAG.json 2> $O/bf_$TAG.err || { echo BENCH FAILED; tail -5 $O/bf_$TAG.err; exit 1; }
cut -c1-400 $O/bf_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pf_$TAG -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pw-sweep > $R/$O/pf_$TAG.log 2>&1 || { echo PROF FAILED; exit 1; }
echo prof ok
cd $R
timeout -k 10 600 python bench_temporal.py --model all --no-cpu-baseline > $O/temporal_$TAG.jsonl 2> $O/temporal_$TAG.err || { echo TEMPORAL FAILED; tail -5 $O/temporal_$TAG.err; exit 1; }
cut -c1-300 $O/temporal_$TAG.jsonl
timeout -k 10 300 python bench.py --dtype fp16 --no-pw-sweep --no-cpu-baseline > $O/bf16mode_$TAG.json 2> $O/bf16mode_$TAG.err || { echo FP16 BENCH FAILED; exit 1; }
cut -c1-300 $O/bf16mode_$TAG.json
