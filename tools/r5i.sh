#!/bin/bash
# round 5: reader phase trace, and the C5 leg with the one-file projection
mkdir -p gpurun_out
timeout -k 10 180 bash tools/reader_trace.sh > gpurun_out/r5i_reader_trace.txt 2>&1; echo "trace rc=$?"; cat gpurun_out/r5i_reader_trace.txt
timeout -k 10 300 python bench.py --config C5 --steps 5 --warmup 1 --no-cpu-baseline --no-pcie --no-reader --no-index --legs=C5 --out gpurun_out/r5i_bench.json > gpurun_out/r5i_bench.log 2>&1; echo "bench rc=$?"
python3 -c "
import json; d=json.load(open('gpurun_out/r5i_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['k_parse_avg_ms'], d['roofline']['avg_launch_ms']); print(json.dumps(d.get('legs',{}).get('C5',{}).get('one_file')))"
