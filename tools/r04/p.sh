#!/bin/bash
# round-4 call P = call O (TN depth A/B) then the final evidence pass (tools/r04/full.sh p).
R=$GRAFT_REPO_ROOT; cd $R
bash tools/r04/o.sh || exit $?
cd $R
bash tools/r04/full.sh p || exit $?
