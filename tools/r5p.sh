#!/bin/bash
# round 5: k_decode_st event counters (landing waits) of the committed build and the working tree on C2
mkdir -p gpurun_out
for v in _var/base birdnest/audio_amd/lib; do
  BNFLAC_LIB_DIR=/root/repo/$v timeout -k 10 200 python bench.py --config C2 --steps 2 --warmup 1 --legs "" --no-cpu-baseline --no-pcie --no-index --no-reader --stats --out gpurun_out/r5p_stats.json > gpurun_out/r5p_stats.log 2>&1 || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/r5p_stats.json')); s=d['stats']; print('$v', d['roofline']['avg_launch_ms'], {k:s[k] for k in ['fused_chunks','generic_chunks','dma_land_waits','slow_rice','refills','waves']})"
done
