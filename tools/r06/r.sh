#!/bin/bash
# round-6 call R: kernel trace of the ViT train step (bench_temporal.py --model vit, 4 + 2 steps)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/vitprof -o run -- python $R/bench_temporal.py --model vit --steps 4 --warmup 2 --no-cpu-baseline > $O/r_vitprof.log 2>&1 || { echo PROF FAILED; tail -5 $O/r_vitprof.log; exit 1; }
echo prof ok
f=$(ls $O/vitprof/*kernel_stats.csv | head -1); cp $f $O/r_vit_kernel_stats.csv
cut -c1-140 $O/r_vit_kernel_stats.csv | head -24
