#!/bin/bash
# round-5 final evidence (after calls S-Z): tools/r05/full.sh on the committed tree, tag r05f
bash "$GRAFT_REPO_ROOT/tools/r05/full.sh" r05f
