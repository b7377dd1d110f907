#!/bin/bash
# round-6 call K: kernel trace of the bf16 ensemble training step (where the 17.7 ms go)
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/k_pf -o run -- python $R/bench_temporal.py --model ensemble_train --clips 8 --steps 5 --warmup 2 --no-cpu-baseline --ens-dtypes bf16 > $R/$O/k_pf.log 2>&1 || { echo PROF FAILED; tail -5 $R/$O/k_pf.log; exit 1; }
tail -2 $R/$O/k_pf.log | cut -c1-200
