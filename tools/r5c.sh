#!/bin/bash
# round 5: k_parse_wave scalar walk for small partitions -- parse-wave parity tests, C5 A/B
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parse_wave.py tests/test_gpu_c5_flow.py > gpurun_out/r5c_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r5c_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/c5_parse_ab.py > gpurun_out/c5ab2.txt 2>&1; echo "c5ab rc=$?"; cat gpurun_out/c5ab2.txt
BNFLAC_PW_SEG=-1 timeout -k 10 300 python tools/c5_parse_ab.py > gpurun_out/c5ab2_off.txt 2>&1; echo "c5ab off rc=$?"; cat gpurun_out/c5ab2_off.txt
