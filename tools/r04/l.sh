#!/bin/bash
# round-4 call L: the im2col-free stem weight gradient (bit-identity, bench A/B, trace) and an in-model
# A/B of the vgemm fragment schedule (ViT step and ensemble serving on libdfd_hip_xp0/xp1/default).
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r04; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_b0_224_gpu.py tests/test_vgemm_gpu.py -q -k "stem_wgrad_direct or knobs_close or eval_bit_identical or vgemm" --timeout 200 --timeout-method thread > $O/l_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/l_tests.log; grep -E "^FAILED" $O/l_tests.log | head
[ $rc -eq 0 ] || exit 1
for i in 1 2; do for v in 1 0; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-pw-sweep --steps 40 --warmup 5 --tune stem_wg=$v > $O/l_b_wg${v}_$i.json 2>/dev/null || { echo "BENCH stem_wg=$v FAILED"; exit 1; }
  echo "stem_wg=$v $(python -c "import json; print(json.load(open('$O/l_b_wg${v}_$i.json'))['ms_per_step'])")"
done; done
for i in 1 2; do for lib in xp0 xp1 default; do
  if [ $lib = default ]; then unset DFD_HIP_LIB; else export DFD_HIP_LIB=$R/deepfake-video-detection_amd/libdfd_hip_$lib.so; fi
  timeout -k 10 300 python bench_temporal.py --model vit --no-cpu-baseline > $O/l_vit_${lib}_$i.jsonl 2>/dev/null || { echo "VIT $lib FAILED"; exit 1; }
  timeout -k 10 300 python bench_temporal.py --model ensemble --no-cpu-baseline > $O/l_ens_${lib}_$i.jsonl 2>/dev/null || { echo "ENS $lib FAILED"; exit 1; }
  echo "$lib vit $(python -c "import json; print(json.load(open('$O/l_vit_${lib}_$i.jsonl'))['ms_per_step'])") ens $(python -c "import json; print(json.load(open('$O/l_ens_${lib}_$i.jsonl'))['ms_per_step'])")"
done; done
unset DFD_HIP_LIB
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pf_l -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pw-sweep > $R/$O/pf_l.log 2>&1 || { echo PROF FAILED; exit 1; }
echo prof ok
