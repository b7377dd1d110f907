#!/bin/bash
# round-5 call R: the tiled weight gradient's M-split target (DFD_WGRAD_SPLIT_WGS 512 default vs 768 /
# 1024 workgroups) -- interleaved bench A/B
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r05; mkdir -p $O
for i in 1 2 3; do for v in default wg768 wg1024; do
  if [ $v = default ]; then L=""; else L=$R/deepfake-video-detection_amd/libdfd_hip_$v.so; fi
  DFD_HIP_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-pw-sweep > $O/r_bench.json 2> $O/r_bench.err || { echo BENCH FAILED; tail -5 $O/r_bench.err; exit 1; }
  python -c "import json;d=json.load(open('$O/r_bench.json'));print('$v', d['ms_per_step'])"
done; done
