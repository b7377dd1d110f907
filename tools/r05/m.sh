#!/bin/bash
# round-5 call M: ViT weight-gradient GEMM with the split partials reduced inside the launch (op 6 /
# the ViT backward) -- vgemm + ViT tests, then the ViT step A/B against the separate-reduction build
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r05; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -rA -k "tn or determ" \
  tests/test_vgemm_gpu.py tests/test_vit_gcn.py > $O/m_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/m_tests.log; grep -E "^FAILED" $O/m_tests.log | head; grep -E "TN op" $O/m_tests.log | cut -c1-160
[ $rc -eq 0 ] || exit 1
for i in 1 2; do for v in coop sep; do
  if [ $v = coop ]; then L=""; else L=$R/deepfake-video-detection_amd/libdfd_hip_tncoop0.so; fi
  DFD_HIP_LIB=$L timeout -k 10 300 python bench_temporal.py --model vit --no-cpu-baseline > $O/m_vit.json 2> $O/m_vit.err || { echo VIT BENCH FAILED; tail -5 $O/m_vit.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/m_vit.json').read().strip().splitlines()[-1]);print('$v', d['ms_per_step'])"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pf_mvit -o run -- python $R/bench_temporal.py --model vit --no-cpu-baseline --steps 3 --warmup 1 > $R/$O/pf_mvit.log 2>&1 || { echo PROF FAILED; exit 1; }
echo prof ok
