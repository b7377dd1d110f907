#!/bin/bash
# round-4 call F: ViT LayerNorm backward + ResNet-50 eval 1x1 convs on the NT GEMM (tests and lines),
# an ensemble-training trace, then the full evidence pass (tools/r04/full.sh).
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r04; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_vit_gcn.py tests/test_vgemm_gpu.py tests/test_resnet.py -q --timeout 200 --timeout-method thread > $O/f_tests.log 2>&1; rc=$?
echo "vit / vgemm / resnet-eval tests rc=$rc"; tail -2 $O/f_tests.log; grep -E "^FAILED" $O/f_tests.log | head
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench_temporal.py --model vit --no-cpu-baseline > $O/f_vitb.jsonl 2> $O/f_vitb.err || { echo VITB FAILED; tail -5 $O/f_vitb.err; exit 1; }
cut -c1-200 $O/f_vitb.jsonl
timeout -k 10 300 python bench_temporal.py --model ensemble --no-cpu-baseline > $O/f_ens.jsonl 2> $O/f_ens.err || { echo ENS FAILED; tail -5 $O/f_ens.err; exit 1; }
cut -c1-200 $O/f_ens.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pf_enst -o run -- python $R/bench_temporal.py --model ensemble_train --no-cpu-baseline --steps 3 --warmup 1 > $R/$O/pf_enst.log 2>&1 || { echo ENST PROF FAILED; exit 1; }
echo enst prof ok
cd $R
bash tools/r04/full.sh f || exit $?
