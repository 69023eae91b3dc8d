#!/bin/bash
# round 5: adaptive refill wait, same-box A/B: committed build (_var/base) / working tree with
# the lag / working tree with the lag switched off (0x4000000: the register-pressure cost alone)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "stereo or long_rice or full_c2" > gpurun_out/r5lag2_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r5lag2_pytest.log
[ $rc -eq 0 ] || exit $rc
ENVS="BNFLAC_LIB_DIR=/root/repo/_var/base;BNFLAC_LIB_DIR=/root/repo/birdnest/audio_amd/lib;BNFLAC_LIB_DIR=/root/repo/birdnest/audio_amd/lib BNFLAC_ABLATE=0x4000000" CFGS="C2" ROUNDS=2 TAG=ab5lag2 bash tools/ab_env.sh || exit $?
BNFLAC_LIB_DIR=/root/repo/birdnest/audio_amd/lib timeout -k 10 200 python bench.py --config C2 --steps 2 --warmup 1 --legs "" --no-cpu-baseline --no-pcie --no-index --no-reader --stats --out gpurun_out/r5lag2_stats.json > gpurun_out/r5lag2_stats.log 2>&1 || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/r5lag2_stats.json')); s=d['stats']; print('lag', d['roofline']['avg_launch_ms'], {k:s[k] for k in ['dma_land_waits','slow_rice']})"
