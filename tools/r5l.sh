#!/bin/bash
# round 5: bulk parse steps -- parity suites for the stereo kernels, then the C2/C3 bench legs
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r5l_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r5l_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-pcie --no-reader --no-index --legs C3,C4 --out gpurun_out/r5l_bench.json > gpurun_out/r5l_bench.log 2>&1; echo "bench rc=$?"
python - <<PY
import json
d=json.loads(open('gpurun_out/r5l_bench.json').read())
print('C2', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['k_parse_avg_ms'], d['roofline']['frac'], d['bitexact'])
for k,v in d.get('legs',{}).items(): print(k, v['value'], v['roofline']['avg_launch_ms'], v['roofline']['k_parse_avg_ms'], v['roofline']['frac'], v['bitexact'])
PY
