#!/bin/bash
# XCD A/B (force off / force on / per-shape rule) on the depthwise kernels, then the bench-config
# parity tests, the bench and a kernel trace
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 60 tools/access_bw > gpurun_out/access_bw.txt 2>&1 || exit $?
bash tools/kb_var.sh xcd2 dw_ x0 x1 xr > /dev/null || exit $?
echo kbv-done
bash tools/r03/check.sh b tests/test_b0_bench_config_gpu.py tests/test_cnn_lstm.py::test_cnn_lstm_224_vs_oracle tests/test_dp_hip_gpu.py
