#!/bin/bash
# round-6 call AH: fp32 conv variants -- weight-gradient loads two m-steps ahead (libdfd_hip_wpf2.so), the
# 64-wide data gradient on 256 x 64 tiles (libdfd_hip_n64.so): CNN-LSTM tests on each, then the step
# interleaved against the default build
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
L=$R/deepfake-video-detection_amd
for v in wpf2 n64; do
  DFD_HIP_LIB=$L/libdfd_hip_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_cnn_lstm.py > $O/ah_tests_$v.log 2>&1; rc=$?
  echo "$v tests rc=$rc $(tail -1 $O/ah_tests_$v.log)"
  [ $rc -eq 0 ] || exit $rc
done
for i in 1 2; do
  for v in base wpf2 n64; do
    if [ $v = base ]; then LIBV=; else LIBV=$L/libdfd_hip_$v.so; fi
    DFD_HIP_LIB=$LIBV timeout -k 10 300 python bench_temporal.py --model cnnlstm --no-cpu-baseline > $O/ah_${v}$i.json 2> $O/ah_${v}$i.err || { echo "$v FAILED"; tail -5 $O/ah_${v}$i.err; exit 1; }
    echo "$v run $i: $(python -c "import json;print(json.load(open('$O/ah_${v}$i.json'))['ms_per_step'])") ms"
  done
done
