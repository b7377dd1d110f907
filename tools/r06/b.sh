#!/bin/bash
# round-6 call B: depthwise residency experiment (tools/r06/build_occ.sh: grid = 1x / 2x the occupancy
# API's answer), interleaved twice; the SE-split contention test with the 4 s occupier
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
for rep in 1 2; do
  for m in 1 2; do
    timeout -k 10 120 ./tools/kbench_occ$m dw_ > $O/b_occ${m}_$rep.txt 2> $O/b_occ${m}_$rep.err || { echo "KBENCH occ$m FAILED"; tail -5 $O/b_occ${m}_$rep.err; exit 1; }
  done
done
grep -h "occupancy" $O/b_occ1_1.err | sort | uniq -c
paste <(cut -c1-90 $O/b_occ1_1.txt) <(cut -c1-40 $O/b_occ2_1.txt) | head -60
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_se_sync_gpu.py > $O/b_sesync.log 2>&1; rc=$?
grep -E "contended|PASSED|FAILED|Error" $O/b_sesync.log | head; exit $rc
