#!/bin/bash
# round-5 call S: planar LDS image for the stride-2 depthwise forward (DFD_DWF_PLANES 1 default vs 0):
# bit identity across the two builds, kernel times from a kernel trace, interleaved bench A/B
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r05; mkdir -p $O
PL0=$R/deepfake-video-detection_amd/libdfd_hip_pl0.so
timeout -k 10 300 python -u tools/r05/libhash.py > $O/s_hash_pl1.txt 2>&1 || { echo HASH FAILED; tail -5 $O/s_hash_pl1.txt; exit 1; }
DFD_HIP_LIB=$PL0 timeout -k 10 300 python -u tools/r05/libhash.py > $O/s_hash_pl0.txt 2>&1 || { echo HASH0 FAILED; tail -5 $O/s_hash_pl0.txt; exit 1; }
cat $O/s_hash_pl1.txt $O/s_hash_pl0.txt
cd /tmp && export TMPDIR=/tmp
for v in pl1 pl0; do
  if [ $v = pl1 ]; then L=""; else L=$PL0; fi
  DFD_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/s_prof_$v -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pw-sweep > $R/$O/s_prof_$v.log 2>&1 || { echo PROF FAILED; tail -5 $R/$O/s_prof_$v.log; exit 1; }
done
cd $R
for i in 1 2 3; do for v in pl1 pl0; do
  if [ $v = pl1 ]; then L=""; else L=$PL0; fi
  DFD_HIP_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-pw-sweep > $O/s_bench.json 2> $O/s_bench.err || { echo BENCH FAILED; tail -5 $O/s_bench.err; exit 1; }
  python -c "import json;d=json.load(open('$O/s_bench.json'));print('$v', d['ms_per_step'])"
done; done
