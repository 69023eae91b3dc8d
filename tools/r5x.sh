#!/bin/bash
# round 5: conflict-free 6-bit CRC-16 field tables (CRC_LAYOUT 2) -- full GPU suite, then a
# same-box A/B against the committed 11/11/10-bit build (_var/base) on C2 and C3
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r5x_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r5x_pytest.log
[ $rc -eq 0 ] || exit $rc
ENVS="BNFLAC_LIB_DIR=/root/repo/_var/base;BNFLAC_LIB_DIR=/root/repo/birdnest/audio_amd/lib" CFGS="C2 C3" ROUNDS=2 TAG=ab5x bash tools/ab_env.sh
