#!/bin/bash
# round 5: full GPU suite (k_decode_st 32-sample chunks in every layout, k_parse carried ring address), then every leg
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r5f_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r5f_pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "Error\|assert" gpurun_out/r5f_pytest.log | head -100; exit $rc; }
timeout -k 10 400 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-pcie --no-reader --no-index --out gpurun_out/r5f_bench.json > gpurun_out/r5f_bench.log 2>&1; echo "bench rc=$?"
python - <<PY
import json
d=json.loads(open('gpurun_out/r5f_bench.json').read())
print('C2', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['k_parse_avg_ms'], d['roofline']['frac'], d['bitexact'])
for k,v in d.get('legs',{}).items(): print(k, v['value'], v['roofline']['avg_launch_ms'], v['roofline']['k_parse_avg_ms'], v['roofline']['frac'], v['bitexact'])
PY
