#!/bin/bash
# round-4 call K: a kernel trace of the ViT train step (bench_temporal --model vit) on the current tree.
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r04; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pf_vit_k -o run -- python $R/bench_temporal.py --model vit --no-cpu-baseline --steps 5 --warmup 2 > $R/$O/pf_vit_k.log 2>&1 || { echo VIT PROF FAILED; tail -5 $R/$O/pf_vit_k.log; exit 1; }
cut -c1-200 $R/$O/pf_vit_k.log | tail -2
echo vit prof ok
