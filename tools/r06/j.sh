#!/bin/bash
# round-6 call J: bf16 training of the ResNet-50 member (k_rn16.hip): kernel tests vs autograd, trunk vs fp64
# within 3x torch bf16 autocast, the bf16 ensemble step; then the fp16 B0 bench (the GEMM bodies moved into
# gemm_body.h) and the ensemble training lines (fp32 and bf16)
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_resnet_train_gpu.py -k "bf16 or ensemble" > $O/j_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "PASSED|FAILED|Error|bf16 trunk" $O/j_tests.log | head -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-pw-sweep --no-cpu-baseline > $O/j_bench_fp16.json 2> $O/j_bench_fp16.err || { echo BENCH FAILED; tail -5 $O/j_bench_fp16.err; exit 1; }
cut -c1-220 $O/j_bench_fp16.json
timeout -k 10 400 python bench_temporal.py --model ensemble_train --clips 8 --steps 5 --warmup 2 --no-cpu-baseline > $O/j_ens.jsonl 2> $O/j_ens.err || { echo ENS FAILED; tail -5 $O/j_ens.err; exit 1; }
cut -c1-300 $O/j_ens.jsonl
