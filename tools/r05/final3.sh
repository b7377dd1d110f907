#!/bin/bash
# round-5 closing check on the committed tree (after the ViT attention, LayerNorm and weight-cast changes): smoke, every -m gpu test, bench
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r05; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_r05h.log 2>&1 || { echo SMOKE FAILED; tail -5 $O/smoke_r05h.log; exit 1; }
tail -1 $O/smoke_r05h.log
timeout -k 10 1000 python -u -m pytest tests/ -q -m gpu --timeout 300 --timeout-method thread > $O/tf_r05h.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -2 $O/tf_r05h.log; grep -E "^FAILED" $O/tf_r05h.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bf_r05h.json 2> $O/bf_r05h.err || { echo BENCH FAILED; tail -5 $O/bf_r05h.err; exit 1; }
cut -c1-300 $O/bf_r05h.json
timeout -k 10 600 python bench_temporal.py --model all --no-cpu-baseline > $O/vit_r05h.jsonl 2> $O/vit_r05h.err || { echo VIT FAILED; exit 1; }
cut -c1-250 $O/vit_r05h.jsonl
