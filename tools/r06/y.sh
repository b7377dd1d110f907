#!/bin/bash
# round-6 call Y: ViT step A/B of the fragment-pipelined K loop on the 256-wide NT tile too (vg_xp 3)
# (libdfd_hip_xp3.so = vg_xp 3; old = default vg_xp 1)
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_vit_gcn.py tests/test_vgemm_gpu.py > $O/y_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/y_tests.log; grep -E "FAILED" $O/y_tests.log | head
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  DFD_HIP_LIB=$R/deepfake-video-detection_amd/libdfd_hip_xp3.so timeout -k 10 200 python bench_temporal.py --model vit --no-cpu-baseline > $O/y_old$i.json 2> $O/y_old$i.err || { echo OLD FAILED; tail -5 $O/y_old$i.err; exit 1; }
  timeout -k 10 200 python bench_temporal.py --model vit --no-cpu-baseline > $O/y_new$i.json 2> $O/y_new$i.err || { echo NEW FAILED; tail -5 $O/y_new$i.err; exit 1; }
  python -c "import json;a=json.load(open('$O/y_old$i.json'));b=json.load(open('$O/y_new$i.json'));print('old %.3f new %.3f'%(a['ms_per_step'],b['ms_per_step']))"
done
