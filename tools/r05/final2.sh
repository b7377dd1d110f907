#!/bin/bash
# round-5 closing check on the committed tree (after the attention change): smoke, every -m gpu test, bench
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r05; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_r05g.log 2>&1 || { echo SMOKE FAILED; tail -5 $O/smoke_r05g.log; exit 1; }
tail -1 $O/smoke_r05g.log
timeout -k 10 1000 python -u -m pytest tests/ -q -m gpu --timeout 300 --timeout-method thread > $O/tf_r05g.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -2 $O/tf_r05g.log; grep -E "^FAILED" $O/tf_r05g.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bf_r05g.json 2> $O/bf_r05g.err || { echo BENCH FAILED; tail -5 $O/bf_r05g.err; exit 1; }
cut -c1-300 $O/bf_r05g.json
timeout -k 10 300 python bench_temporal.py --model vit --no-cpu-baseline > $O/vit_r05g.jsonl 2> $O/vit_r05g.err || { echo VIT FAILED; exit 1; }
cut -c1-200 $O/vit_r05g.jsonl
