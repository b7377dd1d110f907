#!/bin/bash
# round-6 call AK: kernel trace of the fp32 ensemble training step after the fold convolutions
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ensprof -o run -- python $R/bench_temporal.py --model ensemble_train --clips 8 --steps 3 --warmup 1 --no-cpu-baseline --ens-dtypes fp32 > $O/ak_prof.log 2>&1 || { echo PROF FAILED; tail -5 $O/ak_prof.log; exit 1; }
echo prof ok
