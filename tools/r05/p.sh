#!/bin/bash
# round-5 call P: XCD-aware block order for the 7x7-stage channel-pair depthwise backward (adjacent
# 32-channel groups share 128-B lines: on one XCD the second group's half-lines hit L2) -- bench A/B
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r05; mkdir -p $O
LX=$R/deepfake-video-detection_amd/libdfd_hip_xcd1.so
for i in 1 2 3; do for v in default xcd1; do
  if [ $v = default ]; then L=""; else L=$LX; fi
  DFD_HIP_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-pw-sweep > $O/p_bench.json 2> $O/p_bench.err || { echo BENCH FAILED; tail -5 $O/p_bench.err; exit 1; }
  python -c "import json;d=json.load(open('$O/p_bench.json'));print('$v', d['ms_per_step'])"
done; done
cd /tmp && export TMPDIR=/tmp
DFD_HIP_LIB=$LX timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pf_p -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pw-sweep > $R/$O/pf_p.log 2>&1 || { echo PROF FAILED; exit 1; }
echo prof ok
