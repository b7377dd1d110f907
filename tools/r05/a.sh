#!/bin/bash
# round-5 call A: the new parity checks (stem_occ training step vs fp64, vgemm at the C5 M, ResNet conv
# epilogue fallback), the B0 parity tests with the fused SE-backward finalize, bench A/B (tail_fin),
# host enqueue cost, a kernel trace of the bench step.
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r05; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_b0_224_gpu.py tests/test_b0_parity_gpu.py tests/test_vgemm_gpu.py tests/test_resnet.py::test_rn_conv_kernel_every_shape \
  > $O/a_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "stem_occ 3 vs 2|TN .* at M|FAILED|passed|failed" $O/a_tests.log | tail -40
[ $rc -eq 0 ] || exit 1
for t in 1 0 1 0; do
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pw-sweep --tune tail_fin=$t > $O/a_bench_tf$t.json 2> $O/a_bench.err || { echo BENCH FAILED; tail -5 $O/a_bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/a_bench_tf$t.json'));print('tail_fin=$t', d['ms_per_step'], d['value'])"
done
timeout -k 10 300 python tools/r05/host_time.py > $O/a_host.json 2> $O/a_host.err || { echo HOST FAILED; tail -3 $O/a_host.err; exit 1; }
cat $O/a_host.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pf_a -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pw-sweep > $R/$O/pf_a.log 2>&1 || { echo PROF FAILED; exit 1; }
echo prof ok
