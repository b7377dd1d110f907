#!/bin/bash
# round-4 call J: evidence pass with vg_xp = 3 and stem_occ = 3 as defaults, plus the ViT GEMM shapes.
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r04; mkdir -p $O
bash tools/r04/full.sh j || exit $?
timeout -k 10 300 python tools/vgemm_bench.py 3 > $O/j_vgb.jsonl 2> $O/j_vgb.err || { echo VGB FAILED; tail -5 $O/j_vgb.err; exit 1; }
cut -c1-200 $O/j_vgb.jsonl
