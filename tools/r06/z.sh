#!/bin/bash
# round-6 call Z: the ping-pong 256-wide NT schedule: bit-identity tests, then the ViT GEMM
# microbenchmark ("pp" arm)
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_vgemm_gpu.py > $O/z_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/z_tests.log; grep -E "FAILED|Error" $O/z_tests.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/vgemm_bench.py 5 > $O/z_vgemm.jsonl 2> $O/z_vgemm.err || { echo BENCH FAILED; tail -5 $O/z_vgemm.err; exit 1; }
python -c "
import json
for l in open('$O/z_vgemm.jsonl'):
    d=json.loads(l); print(d['shape'], {k[:-3]:v for k,v in d.items() if k.endswith('_us')})"
