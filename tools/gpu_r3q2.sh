#!/bin/bash
# line-flush variant sw8 (no 64-bit add inside the MAC asm): the debug batch and the SW tests
# with sw8 as the library, then C3 A/B against sw5
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIB=birdnest/audio_amd/lib/libbnflac.so
cp $LIB ab/_main.so && cp ab/sw8.so $LIB
PYTHONPATH=. timeout -k 10 120 python tools/dbg_sw_qf.py; rc=$?
[ $rc -eq 0 ] || { cp ab/_main.so $LIB; exit $rc; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decode_sw.py -m gpu > gpurun_out/pytest_r3q2_sw.log 2>&1; rc=$?
cp ab/_main.so $LIB
echo "sw8 tests rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_r3q2_sw.log | tail -2
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=2 AB_ARGS="--config C3 --legs=" bash tools/ab2.sh sw5 sw8
