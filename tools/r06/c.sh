#!/bin/bash
# round-6 call C: depthwise residency experiment (tools/r06/build_occ.sh: grid = 1x / 2x the occupancy
# API's answer), interleaved twice; the SE-split contention test with the 4 s occupier
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
for rep in 1 2; do
  for m in 1 2; do
    timeout -k 10 120 ./tools/kbench_f16_occ$m dw_ > $O/c_occ${m}_$rep.txt 2> $O/c_occ${m}_$rep.err || { echo "KBENCH occ$m FAILED"; tail -5 $O/c_occ${m}_$rep.err; exit 1; }
  done
done
grep -h "occupancy" $O/c_occ1_1.err | sort | uniq -c
true
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_se_sync_gpu.py > $O/c_sesync.log 2>&1; rc=$?
grep -E "contended|PASSED|FAILED|Error" $O/c_sesync.log | head; exit $rc
