#!/bin/bash
# round-6 call D: A/B of the SE excitation's up-front second-product weight loads (DFD_SE_B2PF 1 = the
# default build vs 0 = libdfd_hip_seb2pf0.so), fp16 bench lines interleaved 3x; then the SE-split
# GPU tests on the default build
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
B="python bench.py --steps 30 --warmup 5 --no-pw-sweep --no-cpu-baseline"
: > $O/d_ab.txt
for rep in 1 2 3; do
  for v in default seb2pf0; do
    if [ $v = default ]; then L=""; else L=$R/deepfake-video-detection_amd/libdfd_hip_$v.so; fi
    DFD_HIP_LIB=$L timeout -k 10 300 $B > $O/d_${v}_$rep.json 2> $O/d_err.txt || { echo "BENCH $v FAILED"; tail -5 $O/d_err.txt; exit 1; }
    echo "$v $(python -c "import json,sys; d=json.load(open('$O/d_${v}_$rep.json')); print(d['ms_per_step'])")" | tee -a $O/d_ab.txt
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/d_pf -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pw-sweep > $R/$O/d_pf.log 2>&1 || { echo PROF FAILED; exit 1; }
echo prof ok
