#!/bin/bash
# PMC wave-cycle split of the dw_bwd kernels in the bench (one pass, SQ counters only)
R=$GRAFT_REPO_ROOT; TAG=${1:-p}; RE=${2:-dw_bwd}
OUT=$R/gpurun_out/pmc_$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  --kernel-include-regex "$RE" --output-format csv -d $OUT/sq -o run -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/sq.log 2>&1 || { echo PMC FAILED; tail -5 $OUT/sq.log; exit 1; }
echo PMC ok
