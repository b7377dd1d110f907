#!/bin/bash
R=$GRAFT_REPO_ROOT; TAG=${1:-v}; cd $R; mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests/test_resnet_train_gpu.py tests/test_pwl_fused_gpu.py tests/test_b0_parity_gpu.py tests/test_b0_bench_config_gpu.py tests/test_b0_224_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1; rc=$?
grep -E "first fused|FAILED|passed|failed" gpurun_out/t_$TAG.log | tail -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 tools/kbench fused 256 > gpurun_out/kb_$TAG.txt 2>&1 || { echo KBENCH FAILED; exit 1; }
cat gpurun_out/kb_$TAG.txt
bash tools/r03/prof.sh $TAG
exit $rc
