#!/bin/bash
# k_decode_sys (BNFLAC_DECODE_SYS=1) against the lane kernels (=0) by copies per step, for the
# auto rule in use_decode_sys: decode launch ms (HIP events), bit-exact flag.
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/sys_crossover.txt; : > $O
for cb in ${CASES:-"C4 8" "C4 16" "C4 32" "C4 48" "C4 64" "C4 96" "C3 8" "C3 16" "C3 32" "C3 64" "C2 16" "C2 32" "C2 64"}; do
  set -- $cb
  for m in 0 1; do
    BNFLAC_DECODE_SYS=$m timeout -k 10 200 python bench.py --config $1 --batches $2 --steps 3 --warmup 1 --legs '' --no-cpu-baseline \
      --no-pcie --no-index --no-reader > gpurun_out/sx_$1_$2_$m.json 2> gpurun_out/sx_$1_$2_$m.err || { echo "fail $cb $m" >> $O; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/sx_$1_$2_$m.json').read().strip().splitlines()[-1])
print('$1 B=$2 sys=$m decode_ms', d['roofline']['avg_launch_ms'], 'step_ms', d['ms_per_step'], 'bitexact', d['bitexact'])" >> $O
  done
done
cat $O
