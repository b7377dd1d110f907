#!/bin/bash
# Round-6 HBM traffic of the fp16 bench step (the C2 headline dtype): the probe (dw_bwd2 blocks.1.0), the
# depthwise backward kernels and every BN-backward apply launch (bn_bwd_apply and the fused finalize +
# apply bn_bwd_apply_fin), from PMC counters in separate passes (kernel trace only).  Each pass runs with
# DFD_SITE_LOG, so the plan writes which layer each attributed launch served, in dispatch order
# (round 5's table assigned the apply launches by a fixed order that the fused finalize had changed).
# Aggregate: python tools/pmc_traffic_r06.py gpurun_out/r06/traffic profiles/r06/traffic.json
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r06/traffic; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
RX="dw_bwd2_kernel|dw_bwd1_kernel|bn_bwd_apply_kernel|bn_bwd_apply_fin_kernel"
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
rm -f $OUT/sites_*.txt
DFD_SITE_LOG=$OUT/sites_fetch.txt timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv -d $OUT/fetch -o run -- \
  $BENCH > $OUT/fetch.log 2>&1 || { echo FETCH FAILED; exit 1; }
DFD_SITE_LOG=$OUT/sites_write.txt timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" --output-format csv -d $OUT/write -o run -- \
  $BENCH > $OUT/write.log 2>&1 || { echo WRITE FAILED; exit 1; }
if [ $RAW = 1 ]; then
  DFD_SITE_LOG=$OUT/sites_raw.txt timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-include-regex "$RX" \
    --output-format csv -d $OUT/raw -o run -- $BENCH > $OUT/raw.log 2>&1 || { echo RAW FAILED; exit 1; }
fi
echo PMC ok
