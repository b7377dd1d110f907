#!/bin/bash
# round-6 call G: PMC traffic of the fp16 step with the plan's own launch-site log (tools/r06/traffic.sh),
# then an fp16 bench line and a kernel trace (launch order of the median step for the late-stage table)
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 900 bash tools/r06/traffic.sh > $O/g_traffic.log 2>&1 || { echo TRAFFIC FAILED; tail -5 $O/g_traffic.log; exit 1; }
tail -3 $O/g_traffic.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-pw-sweep --no-cpu-baseline > $O/g_bench_fp16.json 2> $O/g_bench_fp16.err || { echo BENCH FAILED; tail -5 $O/g_bench_fp16.err; exit 1; }
cut -c1-200 $O/g_bench_fp16.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/g_pf -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pw-sweep > $R/$O/g_pf.log 2>&1 || { echo PROF FAILED; exit 1; }
echo prof ok
