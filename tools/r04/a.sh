#!/bin/bash
# round-4 call A: ResNet-50 training parity after the centred BatchNorm forms; counter list; bench.
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r04
timeout -k 10 400 python -u -m pytest tests/test_resnet_train_gpu.py -x -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/r04/a_rn.log 2>&1; rc=$?
echo "rn tests rc=$rc"; tail -4 gpurun_out/r04/a_rn.log
[ $rc -le 1 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/r04/counters.txt 2>&1; echo "list rc=$?"
cd $R
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pw-sweep > gpurun_out/r04/a_bench.json 2> gpurun_out/r04/a_bench.err || { echo BENCH FAILED; tail -5 gpurun_out/r04/a_bench.err; exit 1; }
cut -c1-300 gpurun_out/r04/a_bench.json
