#!/bin/bash
# End-of-session evidence: the whole -m gpu suite, smoke(), the default bench line (with CPU
# baseline and the pointwise MFMA sweep), a rocprofv3 kernel-trace/stats run of the bench (no sweep,
# so the trace holds only training steps), then the temporal/serving benches and their profiles.
R=$GRAFT_REPO_ROOT; TAG=${1:-r02b}
cd $R; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/ -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -2 gpurun_out/t_$TAG.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo SMOKE FAILED; tail gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 500 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-300 gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pw-sweep > $R/gpurun_out/prof_$TAG.log 2>&1 || { echo PROF FAILED; exit 1; }
echo PROF ok
cd $R
bash tools/temporal_round.sh $TAG
