#!/bin/bash
# round-4 call R: the row-per-thread ResNet-50 stem im2col: ResNet / serving tests, the serving line
# and its trace.
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r04; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_resnet.py tests/test_serving.py tests/test_resnet_train_gpu.py tests/test_mbconv7_gpu.py tests/test_b0_parity_gpu.py tests/test_b0_224_gpu.py -q -m gpu --timeout 200 --timeout-method thread > $O/r_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/r_tests.log; grep -E "^FAILED" $O/r_tests.log | head; [ $rc -eq 0 ] || exit 1
for i in 1 2; do timeout -k 10 300 python bench_temporal.py --model ensemble --no-cpu-baseline > $O/r_ens_$i.jsonl 2>/dev/null || { echo ENS FAILED; exit 1; }
  echo "ens $(python -c "import json; d=json.load(open('$O/r_ens_$i.jsonl')); print(d['ms_per_step'], d['value'], d.get('b0_only'))")"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pf_ens_r -o run -- python $R/bench_temporal.py --model ensemble --no-cpu-baseline --steps 5 --warmup 2 > $R/$O/pf_ens_r.log 2>&1 || { echo ENS PROF FAILED; exit 1; }
echo ens prof ok
