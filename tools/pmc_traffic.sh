#!/bin/bash
# HBM traffic of the bench's probed launch (dw_fwd blocks.1.0) from PMC counters, per the
# MI355X microarch guide: FETCH_SIZE and WRITE_SIZE in separate passes (TCC slots), kernel trace
# only (no sys/runtime traces with --pmc).  Output: gpurun_out/pmc_traffic/{fetch,write}/...
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_traffic
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "dw_fwd_kernel" --output-format csv \
  -d $OUT/fetch -o run -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "dw_fwd_kernel" --output-format csv \
  -d $OUT/write -o run -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/write.log 2>&1
echo PMC $?
