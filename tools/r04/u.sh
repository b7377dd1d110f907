#!/bin/bash
# round-4 call U: ResNet-50 layer1 (Cout 64) on the NT GEMM's 64-wide tile -- tests and the serving
# A/B (libdfd_hip_vg64off = those layers on the implicit-GEMM kernel).
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r04; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_vgemm_gpu.py tests/test_resnet.py tests/test_serving.py -q -m gpu --timeout 200 --timeout-method thread > $O/u_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/u_tests.log; grep -E "^FAILED" $O/u_tests.log | head; [ $rc -eq 0 ] || exit 1
for i in 1 2; do for lib in vg64off default; do
  if [ $lib = default ]; then unset DFD_HIP_LIB; else export DFD_HIP_LIB=$R/deepfake-video-detection_amd/libdfd_hip_$lib.so; fi
  timeout -k 10 300 python bench_temporal.py --model ensemble --no-cpu-baseline > $O/u_ens_${lib}_$i.jsonl 2>/dev/null || { echo "ENS $lib FAILED"; exit 1; }
  echo "$lib ens $(python -c "import json; d=json.load(open('$O/u_ens_${lib}_$i.jsonl')); print(d['ms_per_step'], d['value'])")"
done; done
