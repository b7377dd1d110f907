#!/bin/bash
# round-6 call AQ: the fp32 ReLU backward folded into the BN backward (dfd_rn_bn_train_bwd_relu; no relu_bwd pass
# per BN): ResNet-training tests, then the ensemble training lines (compare calls AL / AN: fp32 39.3-39.6 ms)
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_resnet_train_gpu.py > $O/aq_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/aq_tests.log; grep -E "FAILED|ensemble step" $O/aq_tests.log | cut -c1-200 | head -4
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench_temporal.py --model ensemble_train --clips 8 --steps 5 --warmup 2 --no-cpu-baseline --ens-dtypes fp32,bf16 > $O/aq_new$i.jsonl 2> $O/aq_new$i.err || { echo NEW FAILED; tail -3 $O/aq_new$i.err; exit 1; }
  cut -c1-150 $O/aq_new$i.jsonl
done
