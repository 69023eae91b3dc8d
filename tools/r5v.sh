#!/bin/bash
# round 5: k_parse occupancy (LDS padding: 8 KB = 5 waves per SIMD, 10 KB = 4, 13 KB = 3) on C2 / C3 / C4,
# after the parity suite on the current build
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r5v_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r5v_pytest.log
[ $rc -eq 0 ] || exit $rc
ENVS="BNFLAC_PARSE_LDS_PAD=0;BNFLAC_PARSE_LDS_PAD=2048;BNFLAC_PARSE_LDS_PAD=5376" CFGS="C2 C3 C4" ROUNDS=1 TAG=ab5v bash tools/ab_env.sh
