#!/bin/bash
# round-6 call AG: kernel trace of the CNNLSTMHybrid train step after the conv change
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/clprof -o run -- python $R/bench_temporal.py --model cnnlstm --steps 3 --warmup 1 --no-cpu-baseline > $O/ag_clprof.log 2>&1 || { echo PROF FAILED; tail -5 $O/ag_clprof.log; exit 1; }
echo prof ok
