#!/bin/bash
# round-4 call H: the evidence pass on the current tree (tools/r04/full.sh: smoke, every -m gpu test,
# bench line, kernel trace, temporal / serving lines), the ViT GEMM shapes with both NT tile widths,
# and a kernel trace of the bench with the stem at 3 workgroups per CU.
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r04; mkdir -p $O
bash tools/r04/full.sh h || exit $?
timeout -k 10 300 python tools/vgemm_bench.py 3 > $O/h_vgb.jsonl 2> $O/h_vgb.err || { echo VGB FAILED; tail -5 $O/h_vgb.err; exit 1; }
cut -c1-300 $O/h_vgb.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pf_h_stem3 -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pw-sweep --tune stem_occ=3 > $R/$O/pf_h_stem3.log 2>&1 || { echo PROF FAILED; exit 1; }
echo stem3 prof ok
