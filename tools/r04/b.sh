#!/bin/bash
# round-4 call B: the full evidence pass (tools/r04/full.sh), a kernel trace of the ViT train step, and
# the PMC traffic passes (tools/r04/traffic.sh).
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r04; mkdir -p $O
bash tools/r04/full.sh ${1:-b} || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pf_vit -o run -- python $R/bench_temporal.py --model vit --no-cpu-baseline --steps 5 --warmup 2 > $R/$O/pf_vit.log 2>&1 || { echo VIT PROF FAILED; exit 1; }
echo vit prof ok
cd $R
bash tools/r04/traffic.sh || exit $?
