#!/bin/bash
# round-6 call F: the whole GPU suite (incl. the fp64-anchored 224^2 bounds that have not run yet) and smoke
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 1050 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/ > $O/f_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -cE "PASSED" $O/f_tests.log; grep -E "FAILED|Error|passed|failed" $O/f_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/f_smoke.log 2>&1 || { echo SMOKE FAILED; tail -5 $O/f_smoke.log; exit 1; }
tail -3 $O/f_smoke.log
