#!/bin/bash
# kbench A/B experiments in one call: dw fwd prefetch + dw XCD variants (interleaved), then stream-vs-tiled pw
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
bash tools/kb_var.sh pf dw_fwd p0 p1 > /dev/null || exit $?
bash tools/kb_var.sh xcd dw_ x0 x1 > /dev/null || exit $?
bash tools/r03/kt2.sh || exit $?
echo multi-done
