#!/bin/bash
# round-5 call D: A/B of the launch-fusion bits (tail_fin: 1 SE-bwd finalize, 2 split excitation,
# 4 BN-bwd finalize in the apply pass, 8 forward finalize in the consumer) and of the single-call
# backward (segment flushes batched when no hook waits); kernel trace of the default
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r05; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_b0_parity_gpu.py tests/test_b0_224_gpu.py -k "not knobs_close" > $O/d_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/d_tests.log; grep -E "^FAILED" $O/d_tests.log | head
[ $rc -eq 0 ] || exit 1
for i in 1 2; do for v in 1 9 5 3 15; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-pw-sweep --tune tail_fin=$v > $O/d_bench.json 2> $O/d_bench.err || { echo BENCH FAILED; tail -5 $O/d_bench.err; exit 1; }
  python -c "import json;d=json.load(open('$O/d_bench.json'));print('tail_fin=$v', d['ms_per_step'])"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pf_d -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pw-sweep --tune tail_fin=9 > $R/$O/pf_d.log 2>&1 || { echo PROF FAILED; exit 1; }
echo prof ok
