#!/bin/bash
# round-5 call F: the fused 16-bit kernels (streaming / weight-panel 1x1, fused projection and fold
# backward) now also in fp16 -- tests of both dtypes, bf16 vs fp16 benches, fp16 kernel trace
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r05; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -rA \
  tests/test_pw_kernels.py tests/test_pwl_fused_gpu.py tests/test_b0_224_gpu.py tests/test_b0_bench_config_gpu.py \
  tests/test_b0_parity_gpu.py tests/test_train_step_gpu.py > $O/f_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/f_tests.log; grep -E "^FAILED" $O/f_tests.log | head
grep -E "outside \(10|outside bound|fold fused" $O/f_tests.log | cut -c1-220
[ $rc -eq 0 ] || exit 1
for i in 1 2; do for d in bf16 fp16; do
  timeout -k 10 300 python bench.py --dtype $d --no-cpu-baseline --no-pw-sweep > $O/f_bench_$d.json 2> $O/f_bench.err || { echo BENCH FAILED; tail -5 $O/f_bench.err; exit 1; }
  python -c "import json;d=json.load(open('$O/f_bench_$d.json'));print('$d', d['ms_per_step'], d['loss_scaler'], d['roofline']['achieved'] if d.get('roofline') else None)"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pf_f16 -o run -- python $R/bench.py --dtype fp16 --steps 10 --warmup 3 --no-cpu-baseline --no-pw-sweep > $R/$O/pf_f16.log 2>&1 || { echo PROF FAILED; exit 1; }
echo prof ok
