#!/bin/bash
# round-6 call AC: kernel trace of the ViT train step after the side-stream / attention changes
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/vitprof2 -o run -- python $R/bench_temporal.py --model vit --steps 4 --warmup 2 --no-cpu-baseline > $O/ac_vitprof.log 2>&1 || { echo PROF FAILED; tail -5 $O/ac_vitprof.log; exit 1; }
echo prof ok
