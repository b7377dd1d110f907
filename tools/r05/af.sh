#!/bin/bash
# round-5 call AF: ViT LayerNorm forward with 2 rows per wave (loads of both issued first, default)
# vs 1 row per wave (lnf1 build)
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r05; mkdir -p $O
OLD=$R/deepfake-video-detection_amd/libdfd_hip_lnf1.so
timeout -k 10 300 python -u tools/r05/vit_hash.py > $O/af_hash_new.txt 2>&1 || { echo HASH FAILED; tail -5 $O/af_hash_new.txt; exit 1; }
DFD_HIP_LIB=$OLD timeout -k 10 300 python -u tools/r05/vit_hash.py > $O/af_hash_old.txt 2>&1 || { echo HASH0 FAILED; tail -5 $O/af_hash_old.txt; exit 1; }
grep -h feats $O/af_hash_new.txt $O/af_hash_old.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_vit_gcn.py > $O/af_tests.txt 2>&1 || { echo TESTS FAILED; tail -30 $O/af_tests.txt; exit 1; }
tail -1 $O/af_tests.txt
for i in 1 2; do for v in new old; do
  if [ $v = new ]; then L=""; else L=$OLD; fi
  DFD_HIP_LIB=$L timeout -k 10 300 python bench_temporal.py --model vit --no-cpu-baseline > $O/af_vit.json 2> $O/af_vit.err || { echo BENCH FAILED; tail -5 $O/af_vit.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/af_vit.json').read().splitlines()[-1]);print('$v', d['ms_per_step'])"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/af_prof -o run -- python3 $R/bench_temporal.py --model vit --steps 3 --warmup 1 --no-cpu-baseline > $R/$O/af_prof.log 2>&1 || { echo PROF FAILED; tail -5 $R/$O/af_prof.log; exit 1; }
grep -h "ln_fwd" $R/$O/af_prof/run_kernel_stats.csv | cut -d, -f1-4
