#!/bin/bash
# round-6 call I: the conv_pw data + weight gradient pair as one launch (knob pw_pair): bit-identity on
# the 224^2 step, the probe (pair vs serial vs two streams), then the in-process A/B on the fp16 bench step
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  "tests/test_b0_224_gpu.py::test_pw_pair_bit_identical" > $O/i_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "PASSED|FAILED|Error" $O/i_tests.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/pair_probe > $O/i_probe.txt 2>&1 || { echo PROBE FAILED; tail -3 $O/i_probe.txt; exit 1; }
cat $O/i_probe.txt
timeout -k 10 400 python -u tools/ab_bench.py pw_pair 0 1 2 --rounds 6 --steps 5 > $O/i_ab.txt 2>&1 || { echo AB FAILED; tail -5 $O/i_ab.txt; exit 1; }
grep pw_pair $O/i_ab.txt
