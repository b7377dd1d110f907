#!/bin/bash
# round-5 call B: SE-backward finalize fusion, unrolled operand loads; A/B tail_fin 1 / 0 and the
# write-through (no fence) tail protocol build (libdfd_hip_wt.so)
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r05; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_b0_parity_gpu.py tests/test_b0_bench_config_gpu.py tests/test_b0_224_gpu.py > $O/b_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/b_tests.log; grep -E "^FAILED" $O/b_tests.log | head
[ $rc -eq 0 ] || exit 1
DFD_HIP_LIB=$R/deepfake-video-detection_amd/libdfd_hip_wt.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_b0_parity_gpu.py > $O/b_tests_wt.log 2>&1; rc=$?
echo "wt tests rc=$rc"; tail -2 $O/b_tests_wt.log
[ $rc -eq 0 ] || exit 1
for i in 1 2; do
for v in tf1 tf0 wt; do
  case $v in tf1) E=""; A="--tune tail_fin=1";; tf0) E=""; A="--tune tail_fin=0";; wt) E="DFD_HIP_LIB=$R/deepfake-video-detection_amd/libdfd_hip_wt.so"; A="--tune tail_fin=1";; esac
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-pw-sweep $A > $O/b_bench_$v.json 2> $O/b_bench.err || { echo BENCH FAILED; tail -5 $O/b_bench.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b_bench_$v.json'));print('$v', d['ms_per_step'])"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pf_b -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pw-sweep > $R/$O/pf_b.log 2>&1 || { echo PROF FAILED; exit 1; }
echo prof ok
