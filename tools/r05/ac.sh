#!/bin/bash
# round-5 call AC: LayerNorm backward -- 2-row prefetch ring + one round of co-resident workgroups (default)
# vs 1 row + one round (pf1) vs 1 row + 1024 workgroups (pf1g1024 = the previous kernel's schedule)
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r05; mkdir -p $O
L=$R/deepfake-video-detection_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_vit_gcn.py > $O/ac_tests.txt 2>&1 || { echo TESTS FAILED; tail -30 $O/ac_tests.txt; exit 1; }
tail -1 $O/ac_tests.txt
for i in 1 2; do for v in pf2 pf1 pf1g1024; do
  if [ $v = pf2 ]; then LIB=""; else LIB=$L/libdfd_hip_$v.so; fi
  DFD_HIP_LIB=$LIB timeout -k 10 300 python bench_temporal.py --model vit --no-cpu-baseline > $O/ac_vit.json 2> $O/ac_vit.err || { echo BENCH FAILED; tail -5 $O/ac_vit.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/ac_vit.json').read().splitlines()[-1]);print('$v', d['ms_per_step'])"
done; done
cd /tmp && export TMPDIR=/tmp
for v in pf2 pf1g1024; do
  if [ $v = pf2 ]; then LIB=""; else LIB=$L/libdfd_hip_$v.so; fi
  DFD_HIP_LIB=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/ac_prof_$v -o run -- python3 $R/bench_temporal.py --model vit --steps 3 --warmup 1 --no-cpu-baseline > $R/$O/ac_prof_$v.log 2>&1 || { echo PROF FAILED; tail -5 $R/$O/ac_prof_$v.log; exit 1; }
  echo $v; grep -h "ln_bwd\|ln_fwd\|reduce_slabs_kernel" $R/$O/ac_prof_$v/run_kernel_stats.csv | cut -d, -f1-4
done
