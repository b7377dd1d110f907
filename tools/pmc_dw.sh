cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
run() { timeout -k 10 240 rocprofv3 --pmc $2 --output-format csv -d $R/gpurun_out/pmc/$1 -o run -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc/$1.log 2>&1; }
mkdir -p $R/gpurun_out/pmc
run p1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU" && \
run p2 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY" && \
run p3 "FETCH_SIZE" && run p4 "WRITE_SIZE" && run p5 "SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
echo done $?
