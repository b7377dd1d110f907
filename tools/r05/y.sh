#!/bin/bash
# round-5 call Y: stem weight gradient on dense uint8 frames at 3 workgroups per CU (default) vs 2 (swo2
# build): B0 GPU tests, interleaved bench A/B, kernel trace
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r05; mkdir -p $O
OLD=$R/deepfake-video-detection_amd/libdfd_hip_swo2.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_b0_224_gpu.py tests/test_b0_parity_gpu.py tests/test_b0_bench_config_gpu.py > $O/y_tests.txt 2>&1 || { echo TESTS FAILED; tail -30 $O/y_tests.txt; exit 1; }
tail -2 $O/y_tests.txt
for i in 1 2 3; do for v in occ3 occ2; do
  if [ $v = occ3 ]; then L=""; else L=$OLD; fi
  DFD_HIP_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-pw-sweep > $O/y_bench.json 2> $O/y_bench.err || { echo BENCH FAILED; tail -5 $O/y_bench.err; exit 1; }
  python -c "import json;d=json.load(open('$O/y_bench.json'));print('$v', d['ms_per_step'])"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/y_prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pw-sweep > $R/$O/y_prof.log 2>&1 || { echo PROF FAILED; tail -5 $R/$O/y_prof.log; exit 1; }
