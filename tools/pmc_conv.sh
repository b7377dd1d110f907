#!/bin/bash
# PMC passes over the CNN-LSTM train step (bench_temporal.py cnnlstm), one counter group per run
R=$GRAFT_REPO_ROOT; TAG=${1:-c}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/pmc_$TAG
run() { timeout -s KILL 150 rocprofv3 --pmc $2 --output-format csv -d $R/gpurun_out/pmc_$TAG/$1 -o run -- python $R/bench_temporal.py --model cnnlstm --steps 1 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc_$TAG/$1.log 2>&1; }
run p1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" && \
run p2 "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU"
echo done $?
