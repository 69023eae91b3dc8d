#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_decode_sw.py -m gpu > gpurun_out/pytest_r3v_sw.log 2>&1; echo "rc=$?"
grep -E "passed|failed|FAILED" gpurun_out/pytest_r3v_sw.log | head -60
