#!/bin/bash
# round 5: two-deep refill wait in k_decode_st -- stereo parity tests, same-box A/B against the
# committed build, and the committed build's phase timers (tools/_timers) on C2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_decode_classes.py tests/test_gpu_decode_sw.py -m gpu > gpurun_out/r5o_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r5o_pytest.log
[ $rc -eq 0 ] || exit $rc
ENVS="BNFLAC_LIB_DIR=/root/repo/_var/base;BNFLAC_LIB_DIR=/root/repo/birdnest/audio_amd/lib" CFGS="C2 C3" ROUNDS=2 TAG=ab5o bash tools/ab_env.sh || exit $?
BNFLAC_LIB_DIR=/root/repo/tools/_timers timeout -k 10 200 python bench.py --config C2 --steps 2 --warmup 1 --legs "" --no-cpu-baseline --no-pcie --no-index --no-reader --stats --out gpurun_out/r5o_stats.json > gpurun_out/r5o_stats.log 2>&1; echo "stats rc=$?"
python3 -c "
import json; d=json.load(open('gpurun_out/r5o_stats.json')); print(d['stats'])"
