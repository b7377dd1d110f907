#!/bin/bash
# fused attention: kernel tests, ViT model tests, ViT bench + trace
R=$GRAFT_REPO_ROOT; TAG=${1:-f}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v -s --timeout 200 --timeout-method thread tests/test_attention_gpu.py tests/test_vit_gcn.py -m gpu > gpurun_out/t_$TAG.log 2>&1; rc=$?
grep -E "rel err|FAIL|Error|assert|passed|failed" gpurun_out/t_$TAG.log | cut -c1-300 | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench_temporal.py --model vit --no-cpu-baseline > gpurun_out/vit_$TAG.jsonl 2> gpurun_out/vit_$TAG.err || { tail -5 gpurun_out/vit_$TAG.err; exit 1; }
cut -c1-200 gpurun_out/vit_$TAG.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pfv_$TAG -o run -- python $R/bench_temporal.py --model vit --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/pfv_$TAG.log 2>&1 || { echo PROF VIT FAILED; exit 1; }
echo prof vit ok
