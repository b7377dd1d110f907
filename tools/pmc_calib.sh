#!/bin/bash
# PMC traffic of the bench's probed launch (dw_bwd2<bf16,3,8,56,14> of blocks.1.0, the largest
# kernel of the step) and the FETCH_SIZE / WRITE_SIZE calibration it is corrected with
# (tools/fetch_calib: known byte counts in the same 64-B channel-slice access pattern).
# One counter per pass, kernel trace only (MI355X_MICROARCH.md: never with sys/runtime traces).
# Output: gpurun_out/pmc_calib/{calib_<mode>,fetch,write}/...
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_calib
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for m in 0 1 2; do
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/calib_$m -o run -- $R/tools/fetch_calib $m 3 \
    > $OUT/calib_$m.log 2>&1 || { echo "CALIB $m FAILED"; exit 1; }
done
for m in 3 4; do
  timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/calib_$m -o run -- $R/tools/fetch_calib $m 3 \
    > $OUT/calib_$m.log 2>&1 || { echo "CALIB $m FAILED"; exit 1; }
done
echo CALIB ok
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "dw_bwd2_kernel" --output-format csv \
  -d $OUT/fetch -o run -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/fetch.log 2>&1 || { echo FETCH FAILED; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "dw_bwd2_kernel" --output-format csv \
  -d $OUT/write -o run -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/write.log 2>&1 || { echo WRITE FAILED; exit 1; }
echo PMC ok
