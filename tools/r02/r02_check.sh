#!/bin/bash
# Round-2 evidence in one GPU call: the new parity tests (verbose), the whole -m gpu suite, the
# default bench line, a rocprofv3 kernel-trace/stats of the bench, then the PMC calibration passes.
# Test assertion failures (rc 1) do not stop the chain; a crash, abort or time limit does.
R=$GRAFT_REPO_ROOT
TAG=${1:-r02}
cd $R
mkdir -p gpurun_out
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
timeout -k 10 500 python -u -m pytest tests/test_b0_224_gpu.py tests/test_train_step_gpu.py -v -s -m gpu --timeout 240 --timeout-method thread > gpurun_out/tnew_$TAG.log 2>&1; rc=$?
echo "new tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|mismatches|outside|checked" gpurun_out/tnew_$TAG.log | tail -40
ok $rc || exit $rc
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1; rc=$?
echo "all gpu tests rc=$rc"; tail -3 gpurun_out/t_$TAG.log
ok $rc || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_$TAG.log 2>&1 || { echo PROF FAILED; exit 1; }
echo PROF ok
bash $R/tools/pmc_calib.sh
