#!/bin/bash
# A/B of the stride-1 depthwise strip kernel: kbench dw_fwd lines with it off and with each
# candidate set (DFD_STRIP_CFG), then the B0 GPU parity tests.
R=$GRAFT_REPO_ROOT
cd $R
DFD_DW_STRIP=0 timeout -k 10 120 tools/kbench dw_fwd > gpurun_out/kb_strip_off.txt 2>&1 || exit 1
for c in 0 1 2 3; do
  DFD_STRIP_CFG=$c timeout -k 10 120 tools/kbench dw_fwd > gpurun_out/kb_strip_c$c.txt 2>&1 || exit 1
done
timeout -k 10 600 python -m pytest tests/test_b0_parity_gpu.py -x -q > gpurun_out/strip_tests.txt 2>&1
rc=$?
tail -3 gpurun_out/strip_tests.txt
exit $rc
