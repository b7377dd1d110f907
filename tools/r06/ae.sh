#!/bin/bash
# round-6 call AE: ViT / vgemm tests, ViT step A/B of the LayerNorm parameter-gradient reductions on the side stream
# (libdfd_hip_vitprev.so = reductions in place on the caller stream)
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_vit_gcn.py tests/test_vgemm_gpu.py > $O/ae_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/ae_tests.log; grep -E "FAILED" $O/ae_tests.log | head
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  DFD_HIP_LIB=$R/deepfake-video-detection_amd/libdfd_hip_vitprev.so timeout -k 10 200 python bench_temporal.py --model vit --no-cpu-baseline > $O/ae_old$i.json 2> $O/ae_old$i.err || { echo OLD FAILED; tail -5 $O/ae_old$i.err; exit 1; }
  timeout -k 10 200 python bench_temporal.py --model vit --no-cpu-baseline > $O/ae_new$i.json 2> $O/ae_new$i.err || { echo NEW FAILED; tail -5 $O/ae_new$i.err; exit 1; }
  python -c "import json;a=json.load(open('$O/ae_old$i.json'));b=json.load(open('$O/ae_new$i.json'));print('old %.3f new %.3f'%(a['ms_per_step'],b['ms_per_step']))"
done
