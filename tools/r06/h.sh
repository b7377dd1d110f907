#!/bin/bash
# round-6 call H: late-block weight gradients on the side stream with private scratch (wgrad_stream < 0):
# bit-identity against the single-stream step, then an interleaved in-process A/B on the fp16 bench step
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  "tests/test_b0_224_gpu.py::test_wgrad_stream_bit_identical" > $O/h_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "PASSED|FAILED|Error" $O/h_tests.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_bench.py wgrad_stream 0 -50176 -12544 --rounds 6 --steps 5 > $O/h_ab.txt 2>&1 || { echo AB FAILED; tail -5 $O/h_ab.txt; exit 1; }
cat $O/h_ab.txt
