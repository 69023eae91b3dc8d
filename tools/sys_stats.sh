# k_decode_sys phase timers and event counters (ablate 0x100) on C5 (8 files) and a 64-batch C2
# step.  The timers need a variant build: BNFLAC_EXTRA_CFLAGS=-DBNFLAC_PHASE_TIMERS
# BNFLAC_VARIANT_DIR=tools/_timers python -m birdnest.audio_amd.build; LIBS lists variant dirs.
set -u
for lib in ${LIBS:-tools/_timers}; do
  for cfg in "C5 --c5-batch" ${CFG2:-}; do
    BNFLAC_LIB_DIR=$lib BNFLAC_DECODE_SYS=1 timeout -k 10 200 python3 bench.py --config $cfg ${EXTRA:-} --steps 3 --warmup 1 --legs= --no-cpu-baseline --no-pcie --no-index --no-reader --stats > gpurun_out/stx.json 2>&1 || { tail -5 gpurun_out/stx.json; exit 1; }
    python3 -c "
import json
d=json.loads(open('gpurun_out/stx.json').read().strip().splitlines()[-1]); s=d['stats']; print('$lib', '$cfg', '${EXTRA:-}', d['roofline']['avg_launch_ms'], s['sys_cycles'], 'land_waits', s['dma_land_waits'], 'slow', s['slow_rice'], 'refills', s['refills'], 'waves', s['waves'])
"
  done
done
