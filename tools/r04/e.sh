#!/bin/bash
# round-4 call E: conv partial tiles folded every 4 k-steps, vectorised BN+ReLU+max-pool passes:
# CNN-LSTM / ResNet-training tests, the CNN-LSTM and ensemble-training lines, a CNN-LSTM trace.
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r04; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_cnn_lstm.py tests/test_resnet_train_gpu.py -q -s --timeout 200 --timeout-method thread > $O/e_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/e_tests.log; grep -E "worst gradient|FAILED" $O/e_tests.log | cut -c1-200
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python bench_temporal.py --model cnnlstm --no-cpu-baseline > $O/e_cnnb.jsonl 2> $O/e_cnnb.err || { echo CNNB FAILED; tail -5 $O/e_cnnb.err; exit 1; }
cut -c1-200 $O/e_cnnb.jsonl
timeout -k 10 400 python bench_temporal.py --model ensemble_train --no-cpu-baseline > $O/e_enst.jsonl 2> $O/e_enst.err || { echo ENST FAILED; tail -5 $O/e_enst.err; exit 1; }
cut -c1-200 $O/e_enst.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pf_cnn_e -o run -- python $R/bench_temporal.py --model cnnlstm --no-cpu-baseline --steps 3 --warmup 1 > $R/$O/pf_cnn_e.log 2>&1 || { echo CNN PROF FAILED; exit 1; }
echo prof ok
timeout -k 10 400 python -u -m pytest tests/test_vit_gcn.py tests/test_vgemm_gpu.py -q --timeout 200 --timeout-method thread > $O/e_vit.log 2>&1; rc=$?
echo "vit tests rc=$rc"; tail -2 $O/e_vit.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench_temporal.py --model vit --no-cpu-baseline > $O/e_vitb.jsonl 2> $O/e_vitb.err || { echo VITB FAILED; tail -5 $O/e_vitb.err; exit 1; }
cut -c1-200 $O/e_vitb.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pf_enst -o run -- python $R/bench_temporal.py --model ensemble_train --no-cpu-baseline --steps 3 --warmup 1 > $R/$O/pf_enst.log 2>&1 || { echo ENST PROF FAILED; exit 1; }
echo enst prof ok
