set -u
for cfg in "C5 --c5-batch" "C2 --batches 64"; do
  for ab in 0x100 0x800100; do
    BNFLAC_DECODE_SYS=1 BNFLAC_ABLATE=$ab timeout -k 10 200 python3 bench.py --config $cfg --steps 3 --warmup 1 --legs= --no-cpu-baseline --no-pcie --no-index --no-reader --stats > gpurun_out/stx.json 2>&1 || { tail -5 gpurun_out/stx.json; exit 1; }
    python3 -c "
import json
d=json.loads(open('gpurun_out/stx.json').read().strip().splitlines()[-1]); print('$cfg', '$ab', d['roofline']['avg_launch_ms'], d['stats']['sys_cycles'], d['stats']['dma_land_waits'], d['stats']['refills'], d['stats']['waves'])
"
  done
done
