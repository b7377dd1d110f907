#!/bin/bash
# round-5 call Q: whole-step PMC efficiency table (tools/pmc_step.sh: 4 separate counter passes)
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 1000 bash tools/pmc_step.sh r05q > gpurun_out/r05_pmc_q.log 2>&1; rc=$?
tail -3 gpurun_out/r05_pmc_q.log; exit $rc
