#!/bin/bash
# in-process interleaved A/B of plan knobs on the bench step
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_bench.py fold_min_rows 100000 40000 --rounds 6 --steps 5 > gpurun_out/ab3_fold.txt 2>&1 || { tail -5 gpurun_out/ab3_fold.txt; exit 1; }
cat gpurun_out/ab3_fold.txt | tail -2
timeout -k 10 300 python tools/ab_bench.py stream_min_rows 40000 10000 --rounds 6 --steps 5 > gpurun_out/ab3_stream.txt 2>&1 || { tail -5 gpurun_out/ab3_stream.txt; exit 1; }
cat gpurun_out/ab3_stream.txt | tail -2
