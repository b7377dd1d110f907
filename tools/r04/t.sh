#!/bin/bash
# round-4 call T: the ResNet conv1 window prefetch A/B (serving line; libdfd_hip_pf0 = no prefetch),
# then the final evidence pass (tools/r04/full.sh t).
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r04; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_resnet.py tests/test_serving.py -q -m gpu --timeout 200 --timeout-method thread > $O/t_tests.log 2>&1; rc=$?
echo "resnet / serving tests rc=$rc"; tail -1 $O/t_tests.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do for lib in pf0 default; do
  if [ $lib = default ]; then unset DFD_HIP_LIB; else export DFD_HIP_LIB=$R/deepfake-video-detection_amd/libdfd_hip_$lib.so; fi
  timeout -k 10 300 python bench_temporal.py --model ensemble --no-cpu-baseline > $O/t_ens_${lib}_$i.jsonl 2>/dev/null || { echo "ENS $lib FAILED"; exit 1; }
  echo "$lib ens $(python -c "import json; d=json.load(open('$O/t_ens_${lib}_$i.jsonl')); print(d['ms_per_step'], d['value'])")"
done; done
unset DFD_HIP_LIB
bash tools/r04/full.sh t || exit $?
