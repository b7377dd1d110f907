#!/bin/bash
# round-5 call L: (1) the library compiled from source ON the GPU box (hipcc, gfx950) and the B0
# parity tests run against that build; (2) in-model A/B of the bf16 fused projection backward
# without SLP vectorisation; (3) kernel trace of the default bf16 step
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r05; mkdir -p $O /tmp/dfdlib
( while true; do sleep 30; echo "build tick $(date +%T) $(ls /tmp/dfdb 2>/dev/null | wc -l) objects"; done ) & TP=$!
( hipcc --version | head -2; nproc; time timeout -k 10 1200 make -C deepfake-video-detection_amd/csrc BUILD=/tmp/dfdb OUT=/tmp/dfdlib/libdfd_hip.so -j16 ) > $O/l_box_build.log 2>&1; brc=$?
kill $TP
echo "box build rc=$brc"; tail -4 $O/l_box_build.log; ls -la /tmp/dfdlib/
[ $brc -eq 0 ] || exit 1
DFD_HIP_LIB=/tmp/dfdlib/libdfd_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_b0_parity_gpu.py tests/test_train_step_gpu.py > $O/l_box_tests.log 2>&1; rc=$?
echo "tests on the box-built library rc=$rc"; tail -1 $O/l_box_tests.log
python -c "import deepfake_amd._lib as l; print(l.LIB_PATH)" 2>/dev/null
[ $rc -eq 0 ] || exit 1
for i in 1 2; do for v in default noslp; do
  if [ $v = default ]; then L=""; else L=$R/deepfake-video-detection_amd/libdfd_hip_noslp.so; fi
  DFD_HIP_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-pw-sweep > $O/l_bench.json 2> $O/l_bench.err || { echo BENCH FAILED; tail -5 $O/l_bench.err; exit 1; }
  python -c "import json;d=json.load(open('$O/l_bench.json'));print('$v', d['ms_per_step'])"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pf_l -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pw-sweep > $R/$O/pf_l.log 2>&1 || { echo PROF FAILED; exit 1; }
echo prof ok
