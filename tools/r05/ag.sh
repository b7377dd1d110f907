#!/bin/bash
# round-5 call AG: ViT token-embedding backward with 8 images of loads in flight per thread (default)
# vs one image at a time (tbold build)
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r05; mkdir -p $O
OLD=$R/deepfake-video-detection_amd/libdfd_hip_tbold.so
timeout -k 10 300 python -u tools/r05/vit_hash.py > $O/ag_hash_new.txt 2>&1 || { echo HASH FAILED; tail -5 $O/ag_hash_new.txt; exit 1; }
DFD_HIP_LIB=$OLD timeout -k 10 300 python -u tools/r05/vit_hash.py > $O/ag_hash_old.txt 2>&1 || { echo HASH0 FAILED; tail -5 $O/ag_hash_old.txt; exit 1; }
grep -h feats $O/ag_hash_new.txt $O/ag_hash_old.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_vit_gcn.py > $O/ag_tests.txt 2>&1 || { echo TESTS FAILED; tail -30 $O/ag_tests.txt; exit 1; }
tail -1 $O/ag_tests.txt
for i in 1 2; do for v in new old; do
  if [ $v = new ]; then L=""; else L=$OLD; fi
  DFD_HIP_LIB=$L timeout -k 10 300 python bench_temporal.py --model vit --no-cpu-baseline > $O/ag_vit.json 2> $O/ag_vit.err || { echo BENCH FAILED; tail -5 $O/ag_vit.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/ag_vit.json').read().splitlines()[-1]);print('$v', d['ms_per_step'])"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/ag_prof -o run -- python3 $R/bench_temporal.py --model vit --steps 3 --warmup 1 --no-cpu-baseline > $R/$O/ag_prof.log 2>&1 || { echo PROF FAILED; tail -5 $R/$O/ag_prof.log; exit 1; }
grep -h "tokens_bwd" $R/$O/ag_prof/run_kernel_stats.csv | cut -d, -f1-4
