#!/bin/bash
# round-4 call D: CNN-LSTM kernel trace (against profiles/r02/temporal_cnnlstm_kernel_stats.csv).
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r04; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pf_cnn -o run -- python $R/bench_temporal.py --model cnnlstm --no-cpu-baseline --steps 3 --warmup 1 > $R/$O/pf_cnn.log 2>&1 || { echo CNN PROF FAILED; exit 1; }
echo cnn prof ok
