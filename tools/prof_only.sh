#!/bin/bash
# rocprofv3 kernel trace of a short bench run -> gpurun_out/prof_$1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$1 -o run -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_$1.log 2>&1
echo PROF $?
tail -1 $R/gpurun_out/prof_$1.log | cut -c1-200
