#!/bin/bash
# round-4 call M: vg_xp = 1 default, the rational-erf GELU epilogue: tests and an in-model A/B
# (default vs libdfd_hip_erf0 = library erff vs libdfd_hip_xp3 = fragment schedule on both widths).
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r04; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_vgemm_gpu.py tests/test_vit_gcn.py tests/test_resnet.py tests/test_attention_gpu.py -q -m gpu --timeout 200 --timeout-method thread > $O/m_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/m_tests.log; grep -E "^FAILED" $O/m_tests.log | head
[ $rc -eq 0 ] || exit 1
for i in 1 2; do for lib in erf0 xp3 default; do
  if [ $lib = default ]; then unset DFD_HIP_LIB; else export DFD_HIP_LIB=$R/deepfake-video-detection_amd/libdfd_hip_$lib.so; fi
  timeout -k 10 300 python bench_temporal.py --model vit --no-cpu-baseline > $O/m_vit_${lib}_$i.jsonl 2>/dev/null || { echo "VIT $lib FAILED"; exit 1; }
  echo "$lib vit $(python -c "import json; print(json.load(open('$O/m_vit_${lib}_$i.jsonl'))['ms_per_step'])")"
done; done
unset DFD_HIP_LIB
timeout -k 10 300 python bench_temporal.py --model ensemble --no-cpu-baseline > $O/m_ens.jsonl 2>/dev/null || { echo "ENS FAILED"; exit 1; }
echo "ens $(python -c "import json; print(json.load(open('$O/m_ens.jsonl'))['ms_per_step'])")"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pf_vit_m -o run -- python $R/bench_temporal.py --model vit --no-cpu-baseline --steps 5 --warmup 2 > $R/$O/pf_vit_m.log 2>&1 || { echo VIT PROF FAILED; exit 1; }
echo vit prof ok
