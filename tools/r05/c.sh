#!/bin/bash
# round-5 call C: (1) the SE excitation with its first product split over channel slices (tail_fin bit 1,
# slice barrier) -- B0 parity tests first; (2) the tiled weight gradient with two m-steps in flight (knob
# wg_pf) -- kbench per shape, kernel tests and the step A/B (tail_fin 3 / 1, wg_pf 1 / 2)
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r05; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_b0_parity_gpu.py tests/test_b0_bench_config_gpu.py tests/test_b0_224_gpu.py tests/test_pw_kernels.py tests/test_serving.py > $O/c_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/c_tests.log; grep -E "^FAILED" $O/c_tests.log | head
[ $rc -eq 0 ] || exit 1
for pf in 1 2; do timeout -k 10 200 tools/kbench pw_wgrad 256 wg_pf=$pf > $O/c_kb_pf$pf.txt 2>&1 || { echo KB FAILED; tail -3 $O/c_kb_pf$pf.txt; exit 1; }; done
paste <(awk '{print $2, $3}' $O/c_kb_pf1.txt) <(awk '{print $3}' $O/c_kb_pf2.txt) | head -40
for i in 1 2; do for v in "tail_fin=7 wg_pf=1" "tail_fin=3 wg_pf=1" "tail_fin=1 wg_pf=1" "tail_fin=7 wg_pf=2"; do
  A=$(for kv in $v; do echo -n "--tune $kv "; done)
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-pw-sweep $A > $O/c_bench.json 2> $O/c_bench.err || { echo BENCH FAILED; tail -5 $O/c_bench.err; exit 1; }
  python -c "import json;d=json.load(open('$O/c_bench.json'));print('$v', d['ms_per_step'])"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pf_c -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pw-sweep > $R/$O/pf_c.log 2>&1 || { echo PROF FAILED; exit 1; }
echo prof ok
cd $R
timeout -k 10 300 python tools/r05/graph_try.py > $O/c_graph.json 2> $O/c_graph.err; echo "graph rc=$?"; cat $O/c_graph.json; tail -3 $O/c_graph.err
