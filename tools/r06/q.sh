#!/bin/bash
# round-6 call Q: ViT weight-gradient split reductions batched per layer: ViT / vgemm tests, then the
# ViT train step interleaved against the previous build (libdfd_hip_vitprev.so)
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_vit_gcn.py tests/test_vgemm_gpu.py > $O/q_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/q_tests.log; grep -E "FAILED" $O/q_tests.log | head
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  DFD_HIP_LIB=$R/deepfake-video-detection_amd/libdfd_hip_vitprev.so timeout -k 10 200 python bench_temporal.py --model vit --no-cpu-baseline > $O/q_prev$i.json 2> $O/q_prev$i.err || { echo PREV FAILED; tail -5 $O/q_prev$i.err; exit 1; }
  timeout -k 10 200 python bench_temporal.py --model vit --no-cpu-baseline > $O/q_new$i.json 2> $O/q_new$i.err || { echo NEW FAILED; tail -5 $O/q_new$i.err; exit 1; }
  echo "prev: $(cut -c1-150 $O/q_prev$i.json)"; echo "new:  $(cut -c1-150 $O/q_new$i.json)"
done
