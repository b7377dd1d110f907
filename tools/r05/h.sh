#!/bin/bash
# round-5 call H: per-stage backward recompute checks, fp16 at feature-gradient scales 2^15 / 2^20 / 2^24
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r05; mkdir -p $O
for sc in 15 20 24; do
DFD_FP16_SCALE_LOG2=$sc timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu -rA -s \
  tests/test_b0_bench_config_gpu.py -k "per_stage and fp16" > $O/h_tests_$sc.log 2>&1; rc=$?
echo "scale 2^$sc tests rc=$rc"; tail -1 $O/h_tests_$sc.log
grep -E "grad into block|per-stage backward" $O/h_tests_$sc.log | cut -c1-700
done
