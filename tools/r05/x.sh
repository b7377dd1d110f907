#!/bin/bash
# round-5 call X: se_chain split partials with up to 8 slice loads in flight (new) vs one at a time
# (seold build): bit identity, interleaved bench A/B
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r05; mkdir -p $O
OLD=$R/deepfake-video-detection_amd/libdfd_hip_seold.so
timeout -k 10 300 python -u tools/r05/libhash.py > $O/x_hash_new.txt 2>&1 || { echo HASH FAILED; tail -5 $O/x_hash_new.txt; exit 1; }
DFD_HIP_LIB=$OLD timeout -k 10 300 python -u tools/r05/libhash.py > $O/x_hash_old.txt 2>&1 || { echo HASH0 FAILED; tail -5 $O/x_hash_old.txt; exit 1; }
grep feats $O/x_hash_new.txt $O/x_hash_old.txt
for i in 1 2 3; do for v in new old; do
  if [ $v = new ]; then L=""; else L=$OLD; fi
  DFD_HIP_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-pw-sweep > $O/x_bench.json 2> $O/x_bench.err || { echo BENCH FAILED; tail -5 $O/x_bench.err; exit 1; }
  python -c "import json;d=json.load(open('$O/x_bench.json'));print('$v', d['ms_per_step'])"
done; done
