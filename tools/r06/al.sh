#!/bin/bash
# round-6 call AL: the fp32 bottleneck residual add fused into conv1's data-gradient epilogue (no clone / add_
# per block): ResNet-training tests, then the fp32 ensemble training step (compare call AJ's 40.25 ms)
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_resnet_train_gpu.py > $O/al_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/al_tests.log; grep -E "FAILED|ensemble step" $O/al_tests.log | cut -c1-200 | head -4
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench_temporal.py --model ensemble_train --clips 8 --steps 5 --warmup 2 --no-cpu-baseline --ens-dtypes fp32,bf16 > $O/al_new$i.jsonl 2> $O/al_new$i.err || { echo NEW FAILED; tail -3 $O/al_new$i.err; exit 1; }
  cut -c1-150 $O/al_new$i.jsonl
done
