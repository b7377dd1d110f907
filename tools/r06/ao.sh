#!/bin/bash
# round-6 call AO: BN finalize chunk scratch cached per stream: CNN-LSTM / ResNet-training tests, the ensemble
# (fp32, bf16) and CNN-LSTM lines (call AN: bf16 ensemble 18.66 ms with per-call hipMallocAsync; AL: 16.5)
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_cnn_lstm.py tests/test_resnet_train_gpu.py > $O/ao_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/ao_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench_temporal.py --model ensemble_train --clips 8 --steps 8 --warmup 2 --no-cpu-baseline --ens-dtypes bf16,fp32,bf16 > $O/ao_ens.jsonl 2> $O/ao_ens.err || { echo ENS FAILED; tail -3 $O/ao_ens.err; exit 1; }
timeout -k 10 300 python bench_temporal.py --model cnnlstm --no-cpu-baseline > $O/ao_cl.json 2> $O/ao_cl.err || { echo CL FAILED; exit 1; }
cat $O/ao_ens.jsonl $O/ao_cl.json | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['metric'][:40], d['dtype'], d['ms_per_step'])"
