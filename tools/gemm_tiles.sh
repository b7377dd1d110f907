R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pw_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tk_g1.log 2>&1; rc=$?
tail -3 gpurun_out/tk_g1.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/tk_g1.log | head -30; exit $rc; }
for t in -1 0 1 2 3; do timeout -k 10 120 tools/kbench pw 256 stream_min_rows=1000000000000 gemm_tile=$t > gpurun_out/kb_g1_t$t.txt 2>&1 || exit 1; done
echo ok
