#!/bin/bash
# round-6 call AI: the fp32 weight gradient on 16-row wave m-steps (4 workgroups per CU): CNN-LSTM tests,
# then the step interleaved against the 32-row build (libdfd_hip_wms32.so)
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_cnn_lstm.py > $O/ai_tests.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 $O/ai_tests.log)"
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  DFD_HIP_LIB=$R/deepfake-video-detection_amd/libdfd_hip_wms32.so timeout -k 10 300 python bench_temporal.py --model cnnlstm --no-cpu-baseline > $O/ai_old$i.json 2> $O/ai_old$i.err || { echo OLD FAILED; exit 1; }
  timeout -k 10 300 python bench_temporal.py --model cnnlstm --no-cpu-baseline > $O/ai_new$i.json 2> $O/ai_new$i.err || { echo NEW FAILED; exit 1; }
  python -c "import json;a=json.load(open('$O/ai_old$i.json'));b=json.load(open('$O/ai_new$i.json'));print('cnnlstm wms32 %.3f wms16 %.3f'%(a['ms_per_step'],b['ms_per_step']))"
done
