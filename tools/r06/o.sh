#!/bin/bash
# round-6 call O: bf16 ResNet training with the inner ReLU backward folded into the BN backward and one
# weight-pack launch per step: tests (bf16 + ensemble), ensemble lines
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_resnet_train_gpu.py -k "bf16 or ensemble" > $O/o_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/o_tests.log; grep -E "bf16 trunk|FAILED" $O/o_tests.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench_temporal.py --model ensemble_train --clips 8 --steps 8 --warmup 2 --no-cpu-baseline --ens-dtypes bf16,fp32,bf16 > $O/o_ens.jsonl 2> $O/o_ens.err || { echo ENS FAILED; tail -5 $O/o_ens.err; exit 1; }
cut -c1-160 $O/o_ens.jsonl
