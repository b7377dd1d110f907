#!/bin/bash
# round-5 call K: fp16 fused projection backward in its no-SLP translation unit -- determinism
# (kernel harness, whole backward), the 16-bit test suites, bf16 / fp16 benches, fp16 trace
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r05; mkdir -p $O
timeout -k 10 300 ./tools/pwl_det > $O/k_pwl_det.log 2>&1 || { echo PWL_DET FAILED; cat $O/k_pwl_det.log; exit 1; }
grep -c "part diff 0 0 0 0 0" $O/k_pwl_det.log
timeout -k 10 600 python -u tools/r05/fp16_det3.py 32 > $O/k_det3.log 2>&1 || { echo DET3 FAILED; tail $O/k_det3.log; exit 1; }
grep -v amdgpu.ids $O/k_det3.log | cut -c1-120
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -rA \
  tests/test_pw_kernels.py tests/test_pwl_fused_gpu.py tests/test_b0_224_gpu.py tests/test_b0_bench_config_gpu.py \
  tests/test_b0_parity_gpu.py tests/test_train_step_gpu.py > $O/k_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/k_tests.log; grep -E "^FAILED" $O/k_tests.log | head
grep -E "outside \(10|outside bound|fold fused|per-stage backward" $O/k_tests.log | cut -c1-300
[ $rc -eq 0 ] || exit 1
for i in 1 2; do for d in bf16 fp16; do
  timeout -k 10 300 python bench.py --dtype $d --no-cpu-baseline --no-pw-sweep > $O/k_bench_$d.json 2> $O/k_bench.err || { echo BENCH FAILED; tail -5 $O/k_bench.err; exit 1; }
  python -c "import json;d=json.load(open('$O/k_bench_$d.json'));print('$d', d['ms_per_step'], d['loss_scaler'])"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pf_k16 -o run -- python $R/bench.py --dtype fp16 --steps 10 --warmup 3 --no-cpu-baseline --no-pw-sweep > $R/$O/pf_k16.log 2>&1 || { echo PROF FAILED; exit 1; }
echo prof ok
