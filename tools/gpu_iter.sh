#!/bin/bash
# One GPU iteration: new-kernel tests, kbench (streaming vs tiled GEMMs), all GPU tests, bench,
# kernel-trace profile.  Every step time-limited; stops at the first failure.
R=$GRAFT_REPO_ROOT
TAG=${1:-x}
FILTER=${2:-pw}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pw_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tk_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/tk_$TAG.log
[ $rc -ne 0 ] && { echo "KERNEL TESTS FAILED rc=$rc"; grep -E "Error|assert|FAILED" gpurun_out/tk_$TAG.log | head -30; exit $rc; }
timeout -k 10 120 tools/kbench $FILTER > gpurun_out/kb_$TAG.txt 2>&1 || { echo KBENCH FAILED; tail gpurun_out/kb_$TAG.txt; exit 1; }
timeout -k 10 120 tools/kbench $FILTER 256 stream_min_rows=1000000000000 > gpurun_out/kb_${TAG}_tiled.txt 2>&1 || { echo KBENCH2 FAILED; exit 1; }
tail -1 gpurun_out/kb_$TAG.txt; tail -1 gpurun_out/kb_${TAG}_tiled.txt
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/t_$TAG.log
[ $rc -ne 0 ] && { echo "TESTS FAILED rc=$rc"; grep -E "Error|assert|FAILED" gpurun_out/t_$TAG.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_$TAG.log 2>&1
echo PROF $?
