#!/bin/bash
# round 3 (session 2): GPU tests on the new k_decode_st (dot2 zero accumulators, compile-time
# assignment, landing check every other pair), then C2 A/B: HEAD, no-ASFIX, new
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/pytest_r3q.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_r3q.log
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=3 AB_ARGS="--legs=" bash tools/ab2.sh v0 v1n v2
