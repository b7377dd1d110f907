#!/bin/bash
# ResNet training tests + fused-kernel tests + kbench fused rows + bench line
R=$GRAFT_REPO_ROOT; TAG=${1:-rn}; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_resnet_train_gpu.py tests/test_resnet.py tests/test_cnn_lstm.py tests/test_pwl_fused_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1; rc=$?
grep -E "rel |PASSED|FAILED|passed|failed" gpurun_out/t_$TAG.log | tail -45
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 tools/kbench fused 256 > gpurun_out/kb_$TAG.txt 2>&1 || { echo KBENCH FAILED; exit 1; }
cat gpurun_out/kb_$TAG.txt
timeout -k 10 600 python bench.py --no-pw-sweep --no-cpu-baseline > gpurun_out/b_$TAG.json 2> gpurun_out/b_$TAG.err || { echo BENCH FAILED; tail -5 gpurun_out/b_$TAG.err; exit 1; }
cut -c1-300 gpurun_out/b_$TAG.json
exit $rc
