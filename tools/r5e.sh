#!/bin/bash
# round 5: k_decode_st 32-sample chunks + LDS line flush (TU3 = FLACDecoder layout) -- parity + C2 bench
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_decode_classes.py -k "FLACDECODER or flacdecoder or C2 or full or classes or stereo" > gpurun_out/r5e_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r5e_pytest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" gpurun_out/r5e_pytest.log | head -80; exit $rc; }
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-pcie --no-reader --no-index --legs= --out gpurun_out/r5e_bench.json > gpurun_out/r5e_bench.log 2>&1; echo "bench rc=$?"
python - <<PY
import json
d=json.loads(open('gpurun_out/r5e_bench.json').read())
print('C2', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['k_parse_avg_ms'], d['roofline']['frac'], d['bitexact'])
PY
