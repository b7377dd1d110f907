#!/bin/bash
# round-5 call AD: ViT weight casts -- cast and transpose from one read, grid of the largest segment
# (default) vs the wcold build (one segment per output, grid of the largest rows x cols)
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r05; mkdir -p $O
OLD=$R/deepfake-video-detection_amd/libdfd_hip_wcold.so
timeout -k 10 300 python -u tools/r05/vit_hash.py > $O/ad_hash_new.txt 2>&1 || { echo HASH FAILED; tail -5 $O/ad_hash_new.txt; exit 1; }
DFD_HIP_LIB=$OLD timeout -k 10 300 python -u tools/r05/vit_hash.py > $O/ad_hash_old.txt 2>&1 || { echo HASH0 FAILED; tail -5 $O/ad_hash_old.txt; exit 1; }
grep -h feats $O/ad_hash_new.txt $O/ad_hash_old.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_vit_gcn.py > $O/ad_tests.txt 2>&1 || { echo TESTS FAILED; tail -30 $O/ad_tests.txt; exit 1; }
tail -1 $O/ad_tests.txt
for i in 1 2; do for v in new old; do
  if [ $v = new ]; then L=""; else L=$OLD; fi
  DFD_HIP_LIB=$L timeout -k 10 300 python bench_temporal.py --model vit --no-cpu-baseline > $O/ad_vit.json 2> $O/ad_vit.err || { echo BENCH FAILED; tail -5 $O/ad_vit.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/ad_vit.json').read().splitlines()[-1]);print('$v', d['ms_per_step'])"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/ad_prof -o run -- python3 $R/bench_temporal.py --model vit --steps 3 --warmup 1 --no-cpu-baseline > $R/$O/ad_prof.log 2>&1 || { echo PROF FAILED; tail -5 $R/$O/ad_prof.log; exit 1; }
grep -h "wcast" $R/$O/ad_prof/run_kernel_stats.csv | cut -d, -f1-4
