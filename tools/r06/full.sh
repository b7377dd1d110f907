#!/bin/bash
# Round-6 evidence on the current tree: smoke, every -m gpu test, the default bench line (fp16, the C2
# dtype; CPU baseline + pointwise sweep), a bf16 line, a rocprofv3 kernel trace of the bench, the
# temporal / serving / ensemble lines.  usage: tools/r06/full.sh TAG
R=$GRAFT_REPO_ROOT; TAG=${1:-full}; cd $R; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_$TAG.log 2>&1 || { echo SMOKE FAILED; tail -5 $O/smoke_$TAG.log; exit 1; }
tail -1 $O/smoke_$TAG.log
timeout -k 10 1100 python -u -m pytest tests/ -v -m gpu --timeout 300 --timeout-method thread > $O/tf_$TAG.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 $O/tf_$TAG.log; grep -E "^FAILED|FAILED" $O/tf_$TAG.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bf_$TAG.json 2> $O/bf_$TAG.err || { echo BENCH FAILED; tail -5 $O/bf_$TAG.err; exit 1; }
cut -c1-300 $O/bf_$TAG.json
timeout -k 10 300 python bench.py --dtype bf16 --no-pw-sweep --no-cpu-baseline > $O/bbf16_$TAG.json 2> $O/bbf16_$TAG.err || { echo BF16 BENCH FAILED; exit 1; }
cut -c1-200 $O/bbf16_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pf_$TAG -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pw-sweep > $R/$O/pf_$TAG.log 2>&1 || { echo PROF FAILED; exit 1; }
echo prof ok
cd $R
timeout -k 10 700 python bench_temporal.py --model all --no-cpu-baseline > $O/temporal_$TAG.jsonl 2> $O/temporal_$TAG.err || { echo TEMPORAL FAILED; tail -5 $O/temporal_$TAG.err; exit 1; }
cut -c1-200 $O/temporal_$TAG.jsonl
