#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decode_sw.py -m gpu > gpurun_out/pytest_r3u_sw.log 2>&1; rc=$?
echo "sw tests rc=$rc"; tail -3 gpurun_out/pytest_r3u_sw.log
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=2 AB_ARGS="--config C3 --legs=" bash tools/ab2.sh sw3 sw4 sw4:BNFLAC_ABLATE=2
