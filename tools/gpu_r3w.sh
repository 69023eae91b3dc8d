#!/bin/bash
# round 3 end: stage 1 (GPU tests + per-config kernel traces) then stage 2 (PMC + default bench)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r3b STAGE=1 bash tools/final_r3.sh || exit $?
TAG=r3b STAGE=2 bash tools/final_r3.sh || exit $?
