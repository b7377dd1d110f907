#!/bin/bash
# HBM traffic of the bench's probed launch (dw_bwd2 blocks.1.0) and of dw_bwd1 / bn_bwd_apply<bf16,1>
# from PMC counters (MI355X_MICROARCH.md HBM section: FETCH_SIZE and WRITE_SIZE in separate passes,
# kernel trace only, never with sys/runtime traces), plus the FETCH/WRITE calibration on known byte
# counts (tools/fetch_calib) and, when the counters exist, the request-size-aware read count
# (TCC_EA0_RDREQ and its _32B / _64B / _128B classes: FETCH_SIZE tallies 128-B requests at 64 B).  Output: gpurun_out/r05/traffic/...; aggregate with
# python tools/pmc_traffic_r04.py gpurun_out/r05/traffic profiles/r05/traffic.json
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r05/traffic; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
RX="dw_bwd2_kernel|dw_bwd1_kernel|bn_bwd_apply_kernel"
BENCH="python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pw-sweep"
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1
RAW=0; grep -q "TCC_EA0_RDREQ_128B" $OUT/counters.txt && grep -q "TCC_EA0_RDREQ_64B" $OUT/counters.txt && RAW=1
echo "raw request counters: $RAW"
for m in 0 1 2; do
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/calib_f$m -o run -- $R/tools/fetch_calib $m 3 \
    > $OUT/calib_f$m.log 2>&1 || { echo "CALIB f$m FAILED"; exit 1; }
  if [ $RAW = 1 ]; then
    timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv \
      -d $OUT/calib_r$m -o run -- $R/tools/fetch_calib $m 3 > $OUT/calib_r$m.log 2>&1 || { echo "CALIB r$m FAILED"; exit 1; }
  fi
done
for m in 3 4; do
  timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/calib_w$m -o run -- $R/tools/fetch_calib $m 3 \
    > $OUT/calib_w$m.log 2>&1 || { echo "CALIB w$m FAILED"; exit 1; }
done
echo CALIB ok
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv -d $OUT/fetch -o run -- \
  $BENCH > $OUT/fetch.log 2>&1 || { echo FETCH FAILED; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" --output-format csv -d $OUT/write -o run -- \
  $BENCH > $OUT/write.log 2>&1 || { echo WRITE FAILED; exit 1; }
if [ $RAW = 1 ]; then
  timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-include-regex "$RX" \
    --output-format csv -d $OUT/raw -o run -- $BENCH > $OUT/raw.log 2>&1 || { echo RAW FAILED; exit 1; }
fi
echo PMC ok
