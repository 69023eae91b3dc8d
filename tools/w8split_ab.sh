#!/bin/bash
# A/B of the W = 8 instance's split launch (BNF_ABLATE_NO_W8SPLIT = 0x100000: one launch after
# k_decode_st) on C4 at 32 and 256 copies and on C2, interleaved in one process per config.
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/w8split_ab.txt; : > $O
for a in "C4 32" "C4 256" "C2 1024"; do
  set -- $a
  for r in 1 2; do
    timeout -k 10 300 python bench.py --config $1 --batches $2 --steps 5 --warmup 1 --legs '' --no-cpu-baseline --no-pcie \
      --no-index --no-reader --ablate 0x100000,0 > gpurun_out/w8ab_$1_$2_$r.json 2> gpurun_out/w8ab_$1_$2_$r.err || { echo "fail $a" >> $O; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/w8ab_$1_$2_$r.json').read().strip().splitlines()[-1])
print('$1 B=$2 r$r split', d['roofline']['avg_launch_ms'], 'bitexact', d['bitexact'], ' ablations', [(a['ablate'], a['k_decode_ms']) for a in d['ablation']])" >> $O
  done
done
cat $O
