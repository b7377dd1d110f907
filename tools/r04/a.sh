#!/bin/bash
# round-4 call A: ResNet-50 training parity (centred BatchNorm forms); ViT GEMM kernels (k_vgemm.hip)
# parity + timing against hipBLASLt, then the ViT model tests and its train-step line; counter list; bench.
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r04
timeout -k 10 400 python -u -m pytest tests/test_resnet_train_gpu.py -x -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/r04/a_rn.log 2>&1; rc=$?
echo "rn tests rc=$rc"; tail -4 gpurun_out/r04/a_rn.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_vgemm_gpu.py -v -s --timeout 120 --timeout-method thread \
  > gpurun_out/r04/a_vg.log 2>&1; rc=$?
echo "vgemm tests rc=$rc"; tail -4 gpurun_out/r04/a_vg.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/vgemm_bench.py 5 > gpurun_out/r04/a_vgb.jsonl 2> gpurun_out/r04/a_vgb.err || { echo VGB FAILED; tail -5 gpurun_out/r04/a_vgb.err; exit 1; }
cat gpurun_out/r04/a_vgb.jsonl
timeout -k 10 300 python -u -m pytest tests/test_pw_kernels.py -k small_k -v --timeout 120 --timeout-method thread \
  > gpurun_out/r04/a_sk.log 2>&1; rc=$?
echo "small-K tests rc=$rc"; tail -3 gpurun_out/r04/a_sk.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u -m pytest tests/test_b0_224_gpu.py -k 'depthwise_schedule or wgrad_stream or dw_rb_forward' -v -s --timeout 200 --timeout-method thread \
  > gpurun_out/r04/a_pf.log 2>&1; rc=$?
echo "schedule-knob tests rc=$rc"; tail -3 gpurun_out/r04/a_pf.log
[ $rc -eq 0 ] || exit 1
for r in 1 2; do for v in "dw_pf=0" "dw_pf=1" "dw_rb=2" "dw_pf=1 dw_rb=2"; do echo "== $v round $r"; timeout -k 10 120 tools/kbench dw_bwd1 256 $v || exit 1; done; done > gpurun_out/r04/a_kbpf.txt 2>&1 || { echo KBPF FAILED; tail -5 gpurun_out/r04/a_kbpf.txt; exit 1; }
cat gpurun_out/r04/a_kbpf.txt
for r in 1 2; do for v in 0 1; do echo "== dw_rb=$v round $r"; timeout -k 10 120 tools/kbench dw_fwd 256 dw_rb=$v || exit 1; done; done > gpurun_out/r04/a_kbrb.txt 2>&1 || { echo KBRB FAILED; tail -5 gpurun_out/r04/a_kbrb.txt; exit 1; }
cat gpurun_out/r04/a_kbrb.txt
timeout -k 10 400 python -u -m pytest tests/test_vit_gcn.py tests/test_attention_gpu.py -v --timeout 200 --timeout-method thread \
  > gpurun_out/r04/a_vit.log 2>&1; rc=$?
echo "vit tests rc=$rc"; tail -4 gpurun_out/r04/a_vit.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench_temporal.py --model vit --no-cpu-baseline > gpurun_out/r04/a_vitb.jsonl 2> gpurun_out/r04/a_vitb.err || { echo VITB FAILED; tail -5 gpurun_out/r04/a_vitb.err; exit 1; }
cut -c1-300 gpurun_out/r04/a_vitb.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/r04/counters.txt 2>&1; echo "list rc=$?"
cd $R
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pw-sweep > gpurun_out/r04/a_bench.json 2> gpurun_out/r04/a_bench.err || { echo BENCH FAILED; tail -5 gpurun_out/r04/a_bench.err; exit 1; }
cut -c1-300 gpurun_out/r04/a_bench.json
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pw-sweep --tune pw_sk=0 > gpurun_out/r04/a_bench_sk.json 2> gpurun_out/r04/a_bench_sk.err || { echo BENCH SK FAILED; tail -5 gpurun_out/r04/a_bench_sk.err; exit 1; }
cut -c1-300 gpurun_out/r04/a_bench_sk.json
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pw-sweep --tune dw_pf=1 > gpurun_out/r04/a_bench_pf.json 2> gpurun_out/r04/a_bench_pf.err || { echo BENCH PF FAILED; tail -5 gpurun_out/r04/a_bench_pf.err; exit 1; }
cut -c1-300 gpurun_out/r04/a_bench_pf.json
