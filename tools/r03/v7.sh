#!/bin/bash
# Fold-gate check + ensemble-training line + bench/profile.
R=$GRAFT_REPO_ROOT; TAG=${1:-v7}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_pwl_fused_gpu.py tests/test_resnet_train_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1; rc=$?
grep -E "first fused|FAILED|passed|failed" gpurun_out/t_$TAG.log | tail -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench_temporal.py --model ensemble_train > gpurun_out/et_$TAG.jsonl 2> gpurun_out/et_$TAG.err || { echo ET FAILED; tail -20 gpurun_out/et_$TAG.err; exit 1; }
cut -c1-600 gpurun_out/et_$TAG.jsonl
bash tools/r03/prof.sh $TAG
exit $rc
