#!/bin/bash
# round-5 call G: fp16 determinism / fused-vs-unfused per-tensor diagnostics
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r05; mkdir -p $O
timeout -k 10 600 python -u tools/r05/fp16_det.py 32 > $O/g_det.log 2>&1; rc=$?
cat $O/g_det.log | cut -c1-400; exit $rc
