#!/bin/bash
# round-6 call M: A/B of the rn16 128-row tiles' k-step depth (BK 64 default build vs BK 32), interleaved
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_resnet_train_gpu.py -k "bf16" > $O/m_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/m_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in bk64 bk32; do
    lib=deepfake-video-detection_amd/libdfd_hip.so; [ $v = bk32 ] && lib=deepfake-video-detection_amd/libdfd_hip_bk32.so
    DFD_HIP_LIB=$R/$lib timeout -k 10 300 python bench_temporal.py --model ensemble_train --clips 8 --steps 8 --warmup 2 --no-cpu-baseline --ens-dtypes bf16 > $O/m_$v$r.jsonl 2>&1 || { echo FAIL $v; exit 1; }
    echo "$v $r $(grep -o '"ms_per_step": [0-9.]*' $O/m_$v$r.jsonl)"
  done
done
