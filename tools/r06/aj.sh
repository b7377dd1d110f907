#!/bin/bash
# round-6 call AJ: the ResNet-50 fp32 training convolutions (stride 1 and 2, Cin/Cout % 64) on the fp32 tile
# loops with the two-level K / M sum (FOLD): ResNet-training + CNN-LSTM tests, then the fp32 ensemble
# training step interleaved against the conv_gemm build (libdfd_hip_nofold.so)
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_resnet_train_gpu.py tests/test_cnn_lstm.py > $O/aj_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/aj_tests.log; grep -E "FAILED|worst" $O/aj_tests.log | cut -c1-300 | head -6
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  DFD_HIP_LIB=$R/deepfake-video-detection_amd/libdfd_hip_nofold.so timeout -k 10 300 python bench_temporal.py --model ensemble_train --clips 8 --steps 5 --warmup 2 --no-cpu-baseline --ens-dtypes fp32 > $O/aj_old$i.jsonl 2> $O/aj_old$i.err || { echo OLD FAILED; tail -3 $O/aj_old$i.err; exit 1; }
  timeout -k 10 300 python bench_temporal.py --model ensemble_train --clips 8 --steps 5 --warmup 2 --no-cpu-baseline --ens-dtypes fp32 > $O/aj_new$i.jsonl 2> $O/aj_new$i.err || { echo NEW FAILED; tail -3 $O/aj_new$i.err; exit 1; }
  python -c "import json;a=json.loads(open('$O/aj_old$i.jsonl').readline());b=json.loads(open('$O/aj_new$i.jsonl').readline());print('ens fp32 old %.3f new %.3f'%(a['ms_per_step'],b['ms_per_step']))"
done
