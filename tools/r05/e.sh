#!/bin/bash
# round-5 call E: fp16 mode (kernel tests, loss scaler vs GradScaler, fp16 train steps vs the fp32
# oracle), the bf16 suites touched by the 16-bit generalisation, then the tail_fin A/B and an fp16 bench
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r05; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -rA \
  tests/test_train_step_gpu.py tests/test_pw_kernels.py tests/test_b0_224_gpu.py tests/test_b0_bench_config_gpu.py \
  -k "fp16 or gradscaler or half or train_step_224 or golden or late_layers or wgrad" > $O/e_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/e_tests.log; grep -E "^FAILED" $O/e_tests.log | head
grep -E "outside \(10" $O/e_tests.log | cut -c1-160
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --dtype fp16 --no-cpu-baseline --no-pw-sweep > $O/e_bench_fp16.json 2> $O/e_bench_fp16.err || { echo FP16 BENCH FAILED; tail -5 $O/e_bench_fp16.err; exit 1; }
python -c "import json;d=json.load(open('$O/e_bench_fp16.json'));print('fp16', d['ms_per_step'], d['loss_scaler'], d['loss_finite'])"
for i in 1 2; do for v in 15 9 1; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-pw-sweep --tune tail_fin=$v > $O/e_bench.json 2> $O/e_bench.err || { echo BENCH FAILED; tail -5 $O/e_bench.err; exit 1; }
  python -c "import json;d=json.load(open('$O/e_bench.json'));print('tail_fin=$v', d['ms_per_step'])"
done; done
echo done
