#!/bin/bash
# round 5: k_parse_wave per-pass cycle split on the C5 files; the default bench's C5 leg (one-file projection)
mkdir -p gpurun_out
BNFLAC_PW_STATS=1 timeout -k 10 300 python tools/c5_parse_ab.py > gpurun_out/c5ab3_stats.txt 2>&1; echo "c5ab rc=$?"; cat gpurun_out/c5ab3_stats.txt
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-pcie --no-reader --no-index --legs=C5 --out gpurun_out/r5j_bench.json > gpurun_out/r5j_bench.log 2>&1; echo "bench rc=$?"
python3 -c "
import json; d=json.load(open('gpurun_out/r5j_bench.json')); c=d['legs']['C5']; print(c['value'], c['ms_per_step'], c['roofline']['k_parse_avg_ms'], c['roofline']['avg_launch_ms']); print(json.dumps(c.get('one_file')))"
