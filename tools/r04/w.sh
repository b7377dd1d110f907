#!/bin/bash
# round-4 call W: the final tree again (conv1 without the prefetch): every -m gpu test, smoke, serving line.
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r04; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_w.log 2>&1 || { echo SMOKE FAILED; exit 1; }
tail -1 $O/smoke_w.log
timeout -k 10 1000 python -u -m pytest tests/ -q -m gpu --timeout 300 --timeout-method thread > $O/tf_w.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -1 $O/tf_w.log; grep -E "^FAILED" $O/tf_w.log | head; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench_temporal.py --model ensemble --no-cpu-baseline > $O/w_ens.jsonl 2>/dev/null || { echo ENS FAILED; exit 1; }
cut -c1-200 $O/w_ens.jsonl
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pw-sweep > $O/w_bench.json 2>/dev/null || { echo BENCH FAILED; exit 1; }
cut -c1-200 $O/w_bench.json
