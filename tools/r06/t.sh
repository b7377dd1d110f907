#!/bin/bash
# round-6 call T: ViT GEMM microbenchmark (64-wide NT arm), ViT / vgemm tests, ViT step A/B of fc1's
# packed GELU epilogue (libdfd_hip_geluold.so = the scalar form)
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_vit_gcn.py tests/test_vgemm_gpu.py > $O/t_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/t_tests.log; grep -E "FAILED" $O/t_tests.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/vgemm_bench.py 5 > $O/t_vgemm.jsonl 2> $O/t_vgemm.err || { echo BENCH FAILED; tail -5 $O/t_vgemm.err; exit 1; }
python -c "
import json
for l in open('$O/t_vgemm.jsonl'):
    d=json.loads(l); print(d['shape'], {k[:-3]:v for k,v in d.items() if k.endswith('_us')})"
for i in 1 2 3; do
  DFD_HIP_LIB=$R/deepfake-video-detection_amd/libdfd_hip_geluold.so timeout -k 10 200 python bench_temporal.py --model vit --no-cpu-baseline > $O/t_old$i.json 2> $O/t_old$i.err || { echo OLD FAILED; tail -5 $O/t_old$i.err; exit 1; }
  timeout -k 10 200 python bench_temporal.py --model vit --no-cpu-baseline > $O/t_new$i.json 2> $O/t_new$i.err || { echo NEW FAILED; tail -5 $O/t_new$i.err; exit 1; }
  python -c "import json;a=json.load(open('$O/t_old$i.json'));b=json.load(open('$O/t_new$i.json'));print('old %.3f new %.3f'%(a['ms_per_step'],b['ms_per_step']))"
done
