#!/bin/bash
# A/B of two builds of the library on one box: tools/ab_so.sh TAG (tools/ab/libdfd_hip_{old,new}.so),
# interleaved bench runs; the new build is left in place at the end
R=$GRAFT_REPO_ROOT; TAG=${1:-ab}
cd $R; mkdir -p gpurun_out
for v in old new old new old new; do
  cp tools/ab/libdfd_hip_$v.so deepfake-video-detection_amd/libdfd_hip.so
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-pw-sweep > gpurun_out/ab_${TAG}_$v.json 2>gpurun_out/ab_$TAG.err || { tail -5 gpurun_out/ab_$TAG.err; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${TAG}_$v.json)"
done
