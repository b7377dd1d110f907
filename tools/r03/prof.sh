#!/bin/bash
# Bench line + rocprofv3 kernel trace of a short bench run (per-launch durations for the step map).
R=$GRAFT_REPO_ROOT; TAG=${1:-p}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python bench.py --no-pw-sweep > gpurun_out/b_$TAG.json 2> gpurun_out/b_$TAG.err || { echo BENCH FAILED; tail -5 gpurun_out/b_$TAG.err; exit 1; }
cut -c1-400 gpurun_out/b_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pf_$TAG -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pw-sweep > $R/gpurun_out/pf_$TAG.log 2>&1 || { echo PROF FAILED; exit 1; }
echo prof ok
