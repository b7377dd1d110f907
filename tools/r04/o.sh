#!/bin/bash
# round-4 call O: the weight-gradient GEMM with four 32-deep m-step images (libdfd_hip_tn32) -- its
# TN tests on that build, the default build's vgemm tests, and the ViT step A/B.
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r04; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_vgemm_gpu.py tests/test_vit_gcn.py -q --timeout 200 --timeout-method thread > $O/o_tests.log 2>&1; rc=$?
echo "default tests rc=$rc"; tail -1 $O/o_tests.log; [ $rc -eq 0 ] || exit 1
DFD_HIP_LIB=$R/deepfake-video-detection_amd/libdfd_hip_tn32.so timeout -k 10 300 python -u -m pytest tests/test_vgemm_gpu.py tests/test_vit_gcn.py -q --timeout 200 --timeout-method thread > $O/o_tests_tn32.log 2>&1; rc=$?
echo "tn32 tests rc=$rc"; tail -1 $O/o_tests_tn32.log; grep -E "^FAILED" $O/o_tests_tn32.log | head; [ $rc -eq 0 ] || exit 1
for i in 1 2 3; do for lib in tn32 default; do
  if [ $lib = default ]; then unset DFD_HIP_LIB; else export DFD_HIP_LIB=$R/deepfake-video-detection_amd/libdfd_hip_$lib.so; fi
  timeout -k 10 300 python bench_temporal.py --model vit --no-cpu-baseline > $O/o_vit_${lib}_$i.jsonl 2>/dev/null || { echo "VIT $lib FAILED"; exit 1; }
  echo "$lib vit $(python -c "import json; print(json.load(open('$O/o_vit_${lib}_$i.jsonl'))['ms_per_step'])")"
done; done
unset DFD_HIP_LIB
cd /tmp && export TMPDIR=/tmp
DFD_HIP_LIB=$R/deepfake-video-detection_amd/libdfd_hip_tn32.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pf_vit_o -o run -- python $R/bench_temporal.py --model vit --no-cpu-baseline --steps 5 --warmup 2 > $R/$O/pf_vit_o.log 2>&1 || { echo VIT PROF FAILED; exit 1; }
echo vit prof ok
