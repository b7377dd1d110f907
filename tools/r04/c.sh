#!/bin/bash
# round-4 call C: ViT GEMMs with the fused bias gradient and the forward-kept GELU derivative (tests,
# microbench, train-step line, kernel trace), PMC traffic with the request-size counters, and the
# fold_min_rows A/B of the B0 step.
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r04; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_vgemm_gpu.py tests/test_vit_gcn.py tests/test_attention_gpu.py -v --timeout 200 --timeout-method thread > $O/c_vit.log 2>&1; rc=$?
echo "vit/vgemm tests rc=$rc"; tail -3 $O/c_vit.log; grep -E "^FAILED" $O/c_vit.log | head
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/vgemm_bench.py 5 > $O/c_vgb.jsonl 2> $O/c_vgb.err || { echo VGB FAILED; tail -5 $O/c_vgb.err; exit 1; }
timeout -k 10 300 python bench_temporal.py --model vit --no-cpu-baseline > $O/c_vitb.jsonl 2> $O/c_vitb.err || { echo VITB FAILED; tail -5 $O/c_vitb.err; exit 1; }
cut -c1-200 $O/c_vitb.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pf_vit_c -o run -- python $R/bench_temporal.py --model vit --no-cpu-baseline --steps 5 --warmup 2 > $R/$O/pf_vit_c.log 2>&1 || { echo VIT PROF FAILED; exit 1; }
cd $R
bash tools/r04/traffic.sh || exit $?
for v in 100000 0 40000; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-pw-sweep --tune fold_min_rows=$v > $O/c_bench_fold$v.json 2> $O/c_bench_fold$v.err || { echo "BENCH fold $v FAILED"; tail -5 $O/c_bench_fold$v.err; exit 1; }
  echo "fold_min_rows=$v: $(cut -c1-260 $O/c_bench_fold$v.json | grep -o '"ms_per_step": [0-9.]*')"
done
timeout -k 10 400 python -u -m pytest tests/test_cnn_lstm.py tests/test_resnet_train_gpu.py -q --timeout 200 --timeout-method thread > $O/c_cnn.log 2>&1; rc=$?
echo "cnn-lstm / resnet-train tests rc=$rc"; tail -2 $O/c_cnn.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench_temporal.py --model cnnlstm --no-cpu-baseline > $O/c_cnnb.jsonl 2> $O/c_cnnb.err || { echo CNNB FAILED; tail -5 $O/c_cnnb.err; exit 1; }
cut -c1-200 $O/c_cnnb.jsonl
