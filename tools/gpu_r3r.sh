#!/bin/bash
# round 3 (session 2): k_decode_sw tests first, then the whole GPU suite, then A/B: C3 with and
# without k_decode_sw (BNFLAC_ABLATE=0x10000), C2 old vs new k_decode_st
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decode_sw.py -m gpu > gpurun_out/pytest_r3r_sw.log 2>&1; rc=$?
echo "sw tests rc=$rc"; tail -25 gpurun_out/pytest_r3r_sw.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/pytest_r3r.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_r3r.log
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=2 AB_ARGS="--legs=C3" bash tools/ab2.sh sw1 sw1:BNFLAC_ABLATE=0x10000 v0 v1n
