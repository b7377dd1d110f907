#!/bin/bash
# round-6 call AM: the chunked single-pass BN finalize for many centred stat rows: CNN-LSTM + ResNet-training
# tests, then the CNN-LSTM and fp32 ensemble steps interleaved against the previous build (libdfd_hip_bnprev.so)
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_cnn_lstm.py tests/test_resnet_train_gpu.py > $O/am_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/am_tests.log; grep -E "FAILED" $O/am_tests.log | head -4
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  DFD_HIP_LIB=$R/deepfake-video-detection_amd/libdfd_hip_bnprev.so timeout -k 10 300 python bench_temporal.py --model cnnlstm --no-cpu-baseline > $O/am_old$i.json 2> $O/am_old$i.err || { echo OLD FAILED; tail -3 $O/am_old$i.err; exit 1; }
  timeout -k 10 300 python bench_temporal.py --model cnnlstm --no-cpu-baseline > $O/am_new$i.json 2> $O/am_new$i.err || { echo NEW FAILED; tail -3 $O/am_new$i.err; exit 1; }
  python -c "import json;a=json.load(open('$O/am_old$i.json'));b=json.load(open('$O/am_new$i.json'));print('cnnlstm old %.3f new %.3f'%(a['ms_per_step'],b['ms_per_step']))"
done
