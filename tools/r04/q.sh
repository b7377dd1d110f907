#!/bin/bash
# round-4 call Q: kernel traces of the ensemble serving line and of its B0-only arm.
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r04; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pf_ens_q -o run -- python $R/bench_temporal.py --model ensemble --no-cpu-baseline --steps 5 --warmup 2 > $R/$O/pf_ens_q.log 2>&1 || { echo ENS PROF FAILED; tail -5 $R/$O/pf_ens_q.log; exit 1; }
grep -E "^\{" $R/$O/pf_ens_q.log | cut -c1-200
echo ens prof ok
