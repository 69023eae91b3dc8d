#!/bin/bash
# k_decode_sw line flush (sw7): SW tests, every GPU test, C3 A/B against sw5
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decode_sw.py -m gpu > gpurun_out/pytest_r3y_sw.log 2>&1; rc=$?
echo "sw tests rc=$rc"; grep -E "passed|failed|Error" gpurun_out/pytest_r3y_sw.log | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/pytest_r3y.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r3y.log
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=2 AB_ARGS="--config C3 --legs=" bash tools/ab2.sh sw5 sw7
