#!/bin/bash
# round-5 call Z: ViT inference forward without the GELU-derivative store: ViT GPU tests and
# the 128-image forward timing, keep_backward 0 vs 1
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r05; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_vit_gcn.py tests/test_vgemm_gpu.py > $O/z_tests.txt 2>&1 || { echo TESTS FAILED; tail -30 $O/z_tests.txt; exit 1; }
tail -2 $O/z_tests.txt
timeout -k 10 300 python -u tools/r05/vit_inf.py > $O/z_vit_inf.txt 2>&1 || { echo TIMING FAILED; tail -10 $O/z_vit_inf.txt; exit 1; }
grep -v Warning $O/z_vit_inf.txt | tail -3
