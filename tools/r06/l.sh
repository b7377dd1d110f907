#!/bin/bash
# round-6 call L: bf16 ResNet training after the tile choice by tile count (kernel tests, ensemble lines, trace)
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_resnet_train_gpu.py -k "bf16" > $O/l_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/l_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench_temporal.py --model ensemble_train --clips 8 --steps 5 --warmup 2 --no-cpu-baseline --ens-dtypes bf16 > $O/l_ens.jsonl 2> $O/l_ens.err || { echo ENS FAILED; tail -5 $O/l_ens.err; exit 1; }
cut -c1-200 $O/l_ens.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/l_pf -o run -- python $R/bench_temporal.py --model ensemble_train --clips 8 --steps 5 --warmup 2 --no-cpu-baseline --ens-dtypes bf16 > $R/$O/l_pf.log 2>&1 || { echo PROF FAILED; exit 1; }
echo prof ok
