#!/bin/bash
# round-6 call E: the stride-2 depthwise backward with the next tile's staging prefetched (dw_pf bit 1):
# bit-identity tests, kbench (fp16 / bf16) dw_pf 1 vs 3 interleaved, and fp16 bench lines
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
  "tests/test_b0_224_gpu.py::test_dw_bwd2_prefetch_bit_identical" > $O/e_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error" $O/e_tests.log | head; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for pf in 1 3; do
    timeout -k 10 120 ./tools/kbench_f16 dw_bwd2 256 dw_pf=$pf > $O/e_kb16_pf${pf}_$rep.txt 2>&1 || { echo KB FAILED; exit 1; }
    timeout -k 10 120 ./tools/kbench dw_bwd2 256 dw_pf=$pf > $O/e_kb_pf${pf}_$rep.txt 2>&1 || { echo KB FAILED; exit 1; }
  done
done
grep -h "b1 " $O/e_kb16_pf*_*.txt $O/e_kb_pf*_*.txt
B="python bench.py --steps 30 --warmup 5 --no-pw-sweep --no-cpu-baseline"
: > $O/e_ab.txt
for rep in 1 2 3; do
  for pf in 1 3; do
    timeout -k 10 300 $B --tune dw_pf=$pf > $O/e_b_${pf}_$rep.json 2> $O/e_err.txt || { echo "BENCH FAILED"; tail -5 $O/e_err.txt; exit 1; }
    echo "dw_pf=$pf $(python -c "import json; d=json.load(open('$O/e_b_${pf}_$rep.json')); print(d['ms_per_step'], d['roofline']['avg_us'], d['roofline']['frac'])")" | tee -a $O/e_ab.txt
  done
done
