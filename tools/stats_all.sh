#!/bin/bash
# Decode-class mix and k_decode event counters / phase timers per config (debug).
# Phase timers need the variant build: BNFLAC_VARIANT_DIR=tools/_timers
# BNFLAC_EXTRA_CFLAGS=-DBNFLAC_PHASE_TIMERS python -m birdnest.audio_amd.build
set -u
mkdir -p gpurun_out
TAG=${TAG:-stats}
for c in ${CFGS:-C3 C4 C5}; do
  timeout -k 10 120 python tools/class_mix.py $c || exit $?
  BNFLAC_LIB_DIR=${LIBDIR:-tools/_timers} timeout -k 10 200 python bench.py --config $c --steps 2 --warmup 1 --legs "" \
      --no-cpu-baseline --no-pcie --no-index --no-reader --stats > gpurun_out/stats_${TAG}_$c.json || exit $?
  python - <<PY
import json
d = json.loads(open("gpurun_out/stats_${TAG}_$c.json").read().strip().splitlines()[-1])
print("$c", d["value"], d["roofline"]["avg_launch_ms"], d["stats"])
PY
done
