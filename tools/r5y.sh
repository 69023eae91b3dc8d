#!/bin/bash
# round 5: the 11/11/10 CRC layout back as default (sanity: parity suite + C2/C3 against the
# committed build), then the reader's phases (tools/reader_trace.sh)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r5y_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r5y_pytest.log
[ $rc -eq 0 ] || exit $rc
ENVS="BNFLAC_LIB_DIR=/root/repo/_var/base;BNFLAC_LIB_DIR=/root/repo/birdnest/audio_amd/lib" CFGS="C2" ROUNDS=1 TAG=ab5y bash tools/ab_env.sh || exit $?
timeout -k 10 200 bash tools/reader_trace.sh > gpurun_out/r5y_reader.txt 2>&1; echo "reader rc=$?"; cat gpurun_out/r5y_reader.txt
