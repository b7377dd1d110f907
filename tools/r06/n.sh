#!/bin/bash
# round-6 call N: ResNet member gradients written into the detector's flat gradient buffer (no gather /
# scatter copies in the optimizer): the ResNet training tests (fp32 and bf16), the DP / trainer tests,
# and the ensemble training lines
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_resnet_train_gpu.py tests/test_train_step_gpu.py tests/test_resnet.py > $O/n_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/n_tests.log; grep FAILED $O/n_tests.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench_temporal.py --model ensemble_train --clips 8 --steps 8 --warmup 2 --no-cpu-baseline > $O/n_ens.jsonl 2> $O/n_ens.err || { echo ENS FAILED; tail -5 $O/n_ens.err; exit 1; }
cut -c1-200 $O/n_ens.jsonl
