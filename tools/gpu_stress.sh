#!/bin/bash
# Randomised stress on the GPU: N random streams (every generator knob) through the batch API,
# frame index, FLACDecoder layout, reader and stream API; then M corrupted streams through the
# stream API.  usage: N=100 M=50 TAG=r2 bash tools/gpu_stress.sh
set -u
mkdir -p gpurun_out
TAG=${TAG:-stress}
timeout -k 10 ${STRESS_TIMEOUT:-500} python -u tools/stress.py ${N:-100} ${SEED:-11} --index --api --layouts --reader > gpurun_out/stress_${TAG}.log 2>&1; rc=$?; echo "stress rc=$rc"; tail -3 gpurun_out/stress_${TAG}.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 ${STRESS_TIMEOUT:-500} python -u tools/stress.py ${M:-50} ${SEED2:-12} --corrupt > gpurun_out/stress_${TAG}_corrupt.log 2>&1; rc=$?; echo "corrupt rc=$rc"; tail -3 gpurun_out/stress_${TAG}_corrupt.log
