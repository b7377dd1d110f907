#!/bin/bash
# round-4 call N: the final evidence pass on the round's tree (tools/r04/full.sh n).
R=$GRAFT_REPO_ROOT; cd $R
bash tools/r04/full.sh n || exit $?
