#!/bin/bash
# ResNet implicit-GEMM conv: parity tests, ensemble serving bench, then the dw XCD A/B and stream test
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_resnet.py -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/t3_rn.log 2>&1; rc=$?
echo "resnet tests rc=$rc"; grep -E "PASSED|FAILED|Error" gpurun_out/t3_rn.log | tail -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench_temporal.py --model ensemble --no-cpu-baseline > gpurun_out/ens3.json 2> gpurun_out/ens3.err || { echo ENS FAILED; tail -5 gpurun_out/ens3.err; exit 1; }
cat gpurun_out/ens3.json | cut -c1-600
bash tools/r03_multi.sh
