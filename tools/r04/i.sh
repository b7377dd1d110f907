#!/bin/bash
# round-4 call I: the fragment-pipelined vgemm K loop (vg_xp) -- bit-identity tests and the ViT GEMM
# shapes with the xp arm.
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r04; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_vgemm_gpu.py -q --timeout 120 --timeout-method thread > $O/i_tests.log 2>&1; rc=$?
echo "vgemm tests rc=$rc"; tail -2 $O/i_tests.log; grep -E "^FAILED" $O/i_tests.log | head
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/vgemm_bench.py 5 > $O/i_vgb.jsonl 2> $O/i_vgb.err || { echo VGB FAILED; tail -5 $O/i_vgb.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r04/i_vgb.jsonl"):
    d = json.loads(l)
    print(f"{d['shape']:12s} own {d['own_us']:7.1f} xp {d.get('xp_us', 0):7.1f} own128 {d.get('own128_us', 0):7.1f} own256 {d.get('own256_us', 0):7.1f} blaslt {d['blaslt_us']:7.1f}")
PY
