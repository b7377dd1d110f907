#!/bin/bash
# round-5 call N: the depthwise forward embedding the BN1 finalize up to 128 producer stat rows
# (DFD_BNFIN_ROWS=128 build of k_dw_fwd.hip) -- parity on that build, then an interleaved bench A/B
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r05; mkdir -p $O
L128=$R/deepfake-video-detection_amd/libdfd_hip_fin128.so
DFD_HIP_LIB=$L128 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_b0_parity_gpu.py tests/test_b0_224_gpu.py -k "fp32 or bit_reproducible or golden" > $O/n_tests.log 2>&1; rc=$?
echo "tests (fin128 build) rc=$rc"; tail -1 $O/n_tests.log; grep -E "^FAILED" $O/n_tests.log | head
[ $rc -eq 0 ] || exit 1
for i in 1 2 3; do for v in default fin128; do
  if [ $v = default ]; then L=""; else L=$L128; fi
  DFD_HIP_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-pw-sweep > $O/n_bench.json 2> $O/n_bench.err || { echo BENCH FAILED; tail -5 $O/n_bench.err; exit 1; }
  python -c "import json;d=json.load(open('$O/n_bench.json'));print('$v', d['ms_per_step'])"
done; done
