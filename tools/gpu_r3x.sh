#!/bin/bash
# the quad-flush k_decode_sw (sw6: per-MAC asm) on the SW tests, then C3 A/B against sw5
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIB=birdnest/audio_amd/lib/libbnflac.so
cp $LIB ab/_main.so && cp ab/sw6.so $LIB
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_decode_sw.py -m gpu > gpurun_out/pytest_r3x_sw.log 2>&1; rc=$?
cp ab/_main.so $LIB
echo "sw6 tests rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_r3x_sw.log | tail -3
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=2 AB_ARGS="--config C3 --legs=" bash tools/ab2.sh sw5 sw6
