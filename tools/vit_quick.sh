#!/bin/bash
# ViT parity/determinism tests, then the C5 bench line (no CPU baseline)
R=$GRAFT_REPO_ROOT; TAG=${1:-v}
cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_vit_gcn.py tests/test_torch_ops.py -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/tv_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/tv_$TAG.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench_temporal.py --model vit --steps 5 --warmup 2 --no-cpu-baseline
