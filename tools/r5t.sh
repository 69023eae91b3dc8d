#!/bin/bash
# round 5: k_crc_spec (the frames' CRC-16 ahead of the decode) -- full GPU suite, then A/B with
# it switched off (ablation 0x2000000) on C2-C4
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r5t_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r5t_pytest.log
[ $rc -eq 0 ] || exit $rc
ENVS="BNFLAC_ABLATE=0x2000000;BNFLAC_ABLATE=0" CFGS="C2 C3 C4" ROUNDS=1 TAG=ab5r bash tools/ab_env.sh
