#!/bin/bash
# round-5 call I: which knob makes the fp16 backward non-deterministic
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r05; mkdir -p $O
timeout -k 10 600 python -u tools/r05/fp16_det3.py 32 > $O/i_det3.log 2>&1; rc=$?
grep -v amdgpu.ids $O/i_det3.log | cut -c1-400; exit $rc
