#!/bin/bash
# conv GEMM tile change: ResNet training / CNN-LSTM / ResNet parity tests, then the two temporal lines.
R=$GRAFT_REPO_ROOT; TAG=${1:-conv}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_resnet_train_gpu.py tests/test_cnn_lstm.py tests/test_resnet.py tests/test_vit_gcn.py -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/t_$TAG.log; grep -E "FAILED|Error" gpurun_out/t_$TAG.log | head -10
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench_temporal.py --model ensemble_train --no-cpu-baseline > gpurun_out/et_$TAG.jsonl 2> gpurun_out/et_$TAG.err || { echo ET FAILED; tail -5 gpurun_out/et_$TAG.err; exit 1; }
cut -c1-300 gpurun_out/et_$TAG.jsonl
timeout -k 10 400 python -u bench_temporal.py --model cnnlstm --no-cpu-baseline > gpurun_out/cl_$TAG.jsonl 2> gpurun_out/cl_$TAG.err || { echo CL FAILED; tail -5 gpurun_out/cl_$TAG.err; exit 1; }
cut -c1-300 gpurun_out/cl_$TAG.jsonl
exit $rc
