#!/bin/bash
# round-6 call A: the fixes of the first hour -- fused projection backward determinism with SLP on
# (tools/pwl_det once), the SE slice barrier under contention, loss-scaled steps over several flat
# runs, the 224^2 bit-reproducibility and BN forward finalize race checks, then an fp16 and a bf16
# bench line and a kernel trace of the fp16 bench.
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 180 ./tools/pwl_det > $O/a_pwl_det.txt 2>&1 || { echo PWL_DET FAILED; tail -5 $O/a_pwl_det.txt; exit 1; }
cut -c1-150 $O/a_pwl_det.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_se_sync_gpu.py tests/test_train_step_gpu.py "tests/test_b0_224_gpu.py::test_step_224_bit_reproducible" \
  tests/test_b0_bench_config_gpu.py -s > $O/a_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -4 $O/a_tests.log; grep -E "FAILED|contended" $O/a_tests.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-pw-sweep --no-cpu-baseline > $O/a_bench_fp16.json 2> $O/a_bench_fp16.err || { echo BENCH FAILED; tail -5 $O/a_bench_fp16.err; exit 1; }
cut -c1-300 $O/a_bench_fp16.json
timeout -k 10 300 python bench.py --dtype bf16 --steps 20 --warmup 5 --no-pw-sweep --no-cpu-baseline > $O/a_bench_bf16.json 2> $O/a_bench_bf16.err || { echo BENCH16 FAILED; exit 1; }
cut -c1-300 $O/a_bench_bf16.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/a_pf -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pw-sweep > $R/$O/a_pf.log 2>&1 || { echo PROF FAILED; exit 1; }
echo prof ok
