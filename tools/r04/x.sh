#!/bin/bash
# round-4 call X: ViT / vgemm / ResNet tests and smoke on the final tree (vit.cpp width guard).
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r04; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_x.log 2>&1 || { echo SMOKE FAILED; exit 1; }
tail -1 $O/smoke_x.log
timeout -k 10 600 python -u -m pytest tests/test_vit_gcn.py tests/test_vgemm_gpu.py tests/test_attention_gpu.py tests/test_resnet.py tests/test_serving.py -q -m gpu --timeout 200 --timeout-method thread > $O/x_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/x_tests.log; grep -E "^FAILED" $O/x_tests.log | head; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench_temporal.py --model vit --no-cpu-baseline > $O/x_vit.jsonl 2>/dev/null || { echo VIT FAILED; exit 1; }
cut -c1-200 $O/x_vit.jsonl
