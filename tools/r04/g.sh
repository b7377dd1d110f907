#!/bin/bash
# round-4 call G: ResNet-50 bf16 eval 3x3 / strided convolutions on the implicit-conv NT GEMM and the
# SE excitation's batched loads -- tests, the B0 bench line, a kernel trace, the ensemble lines.
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r04; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_vgemm_gpu.py tests/test_vit_gcn.py tests/test_resnet.py tests/test_b0_parity_gpu.py tests/test_b0_bench_config_gpu.py tests/test_serving.py -q -m gpu --timeout 200 --timeout-method thread > $O/g_tests.log 2>&1; rc=$?
echo "resnet / b0 parity / serving tests rc=$rc"; tail -2 $O/g_tests.log; grep -E "^FAILED" $O/g_tests.log | head
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pw-sweep > $O/g_bench.json 2> $O/g_bench.err || { echo BENCH FAILED; tail -5 $O/g_bench.err; exit 1; }
cut -c1-300 $O/g_bench.json
timeout -k 10 300 python bench_temporal.py --model ensemble --no-cpu-baseline > $O/g_ens.jsonl 2> $O/g_ens.err || { echo ENS FAILED; tail -5 $O/g_ens.err; exit 1; }
cut -c1-300 $O/g_ens.jsonl
timeout -k 10 300 python bench_temporal.py --model vit --no-cpu-baseline > $O/g_vit.jsonl 2> $O/g_vit.err || { echo VIT FAILED; tail -5 $O/g_vit.err; exit 1; }
cut -c1-250 $O/g_vit.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pf_g -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pw-sweep > $R/$O/pf_g.log 2>&1 || { echo PROF FAILED; exit 1; }
echo prof ok
cd $R
timeout -k 10 300 python -u -m pytest tests/test_b0_224_gpu.py -q -k "knobs_close or eval_bit_identical" --timeout 200 --timeout-method thread > $O/g_knobs.log 2>&1; echo "knob tests rc=$?"; tail -2 $O/g_knobs.log
for i in 1 2; do for rs in 14 4 5; do echo "== dw2_rs=$rs"; timeout -k 10 120 tools/kbench dw_bwd2 256 dw2_rs=$rs || exit 1; done; done > $O/g_kb_dw2.log 2>&1
grep -E "^==|dw_bwd2" $O/g_kb_dw2.log
for i in 1 2; do for v in 0 3; do echo "== dwf_pf=$v"; timeout -k 10 120 tools/kbench dw_fwd 256 dwf_pf=$v || exit 1; done; done > $O/g_kb_dwf.log 2>&1
grep -E "^==|s2" $O/g_kb_dwf.log
for cfg in "stem_occ=3" "stem_occ=3 dw2_rs=5 dwf_pf=3" "stem_occ=2"; do
  tag=$(echo $cfg | tr ' =' '_-'); args=""; for kv in $cfg; do args="$args --tune $kv"; done
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-pw-sweep --steps 30 --warmup 5 $args > $O/g_ab_$tag.json 2>/dev/null || { echo "AB $cfg FAILED"; exit 1; }
  echo "$cfg $(python -c "import json; d=json.load(open('$O/g_ab_$tag.json')); print(d['ms_per_step'])")"
done
timeout -k 10 300 python tools/vgemm_bench.py 3 > $O/g_vgb.jsonl 2> $O/g_vgb.err || { echo VGB FAILED; tail -5 $O/g_vgb.err; exit 1; }
tail -3 $O/g_vgb.jsonl | cut -c1-250
