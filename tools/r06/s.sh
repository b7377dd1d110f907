#!/bin/bash
# round-6 call S: ViT GEMM shapes, own kernels (incl. the 64-wide NT tile for the 768-wide products) vs hipBLASLt
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 300 python tools/vgemm_bench.py 5 > $O/s_vgemm.jsonl 2> $O/s_vgemm.err || { echo BENCH FAILED; tail -5 $O/s_vgemm.err; exit 1; }
python -c "
import json
for l in open('$O/s_vgemm.jsonl'):
    d=json.loads(l); print(d['shape'], {k:v for k,v in d.items() if k.endswith('_us')})"
