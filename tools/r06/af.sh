#!/bin/bash
# round-6 call AF: fp32 convolutions (CNNLSTMHybrid conv 2..4, the fp32 ResNet-50 training path's stride-1
# layers) on the wide-vector tile loops: CNN-LSTM / ResNet-training / conv tests, then the CNN-LSTM and
# fp32 ensemble-training lines against the previous build (libdfd_hip_convprev.so), interleaved
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_cnn_lstm.py tests/test_resnet_train_gpu.py > $O/af_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/af_tests.log; grep -E "FAILED|Error" $O/af_tests.log | head
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  DFD_HIP_LIB=$R/deepfake-video-detection_amd/libdfd_hip_convprev.so timeout -k 10 300 python bench_temporal.py --model cnnlstm --no-cpu-baseline > $O/af_old$i.json 2> $O/af_old$i.err || { echo OLD FAILED; tail -5 $O/af_old$i.err; exit 1; }
  timeout -k 10 300 python bench_temporal.py --model cnnlstm --no-cpu-baseline > $O/af_new$i.json 2> $O/af_new$i.err || { echo NEW FAILED; tail -5 $O/af_new$i.err; exit 1; }
  python -c "import json;a=json.load(open('$O/af_old$i.json'));b=json.load(open('$O/af_new$i.json'));print('cnnlstm old %.3f new %.3f'%(a['ms_per_step'],b['ms_per_step']))"
done
DFD_HIP_LIB=$R/deepfake-video-detection_amd/libdfd_hip_convprev.so timeout -k 10 300 python bench_temporal.py --model ensemble_train --clips 8 --steps 5 --warmup 2 --no-cpu-baseline --ens-dtypes fp32 > $O/af_eold.jsonl 2> $O/af_eold.err || { echo EOLD FAILED; tail -5 $O/af_eold.err; exit 1; }
timeout -k 10 300 python bench_temporal.py --model ensemble_train --clips 8 --steps 5 --warmup 2 --no-cpu-baseline --ens-dtypes fp32 > $O/af_enew.jsonl 2> $O/af_enew.err || { echo ENEW FAILED; tail -5 $O/af_enew.err; exit 1; }
echo "ens fp32 old $(cut -c1-170 $O/af_eold.jsonl)"; echo "ens fp32 new $(cut -c1-170 $O/af_enew.jsonl)"
