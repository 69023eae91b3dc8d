#!/bin/bash
# k_decode_sw: GPU tests, C3 A/B (sw1: a wait state per MAC, sw2: per older-tap sum), C3 counters + kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decode_sw.py -m gpu > gpurun_out/pytest_r3t_sw.log 2>&1; rc=$?
echo "sw tests rc=$rc"; tail -3 gpurun_out/pytest_r3t_sw.log
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=2 AB_ARGS="--config C3 --legs=" bash tools/ab2.sh sw1 sw2 || exit 1
bash tools/gpu_r3s.sh
