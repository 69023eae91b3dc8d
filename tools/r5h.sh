#!/bin/bash
# round 5: early CRC in half of k_decode_st's waves -- stereo suites, then C2 A/B vs ablations
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_decode_classes.py tests/test_gpu_decode_sys.py > gpurun_out/r5h_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r5h_pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "Error\|assert" gpurun_out/r5h_pytest.log | head -100; exit $rc; }
ENVS="BNFLAC_ABLATE=0;BNFLAC_ABLATE=1" CFGS="C2" ROUNDS=2 TAG=abl6 EXTRA="--batches 512" bash tools/ab_env.sh
