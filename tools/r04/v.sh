#!/bin/bash
# round-4 call V: the evidence pass on the round's final tree (tools/r04/full.sh v).
R=$GRAFT_REPO_ROOT; cd $R
bash tools/r04/full.sh v || exit $?
