#!/bin/bash
# Quick GPU check: every -m gpu test, then a short bench (all legs, no CPU baseline).
set -u
mkdir -p gpurun_out
TAG=${TAG:-quick}
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu ${PYTEST_ARGS:-} > gpurun_out/pytest_$TAG.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_$TAG.log
[ $rc -le 1 ] || exit $rc
[ "${NOBENCH:-0}" = 1 ] && exit 0
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-pcie --no-reader --no-index --out gpurun_out/bench_$TAG.json > gpurun_out/bench_$TAG.log 2>&1; echo "bench rc=$?"
python - <<PY
import json
d=json.loads(open('gpurun_out/bench_$TAG.json').read())
print('C2', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['k_parse_avg_ms'], d['roofline']['frac'], d['bitexact'])
for k,v in d.get('legs',{}).items(): print(k, v['value'], v['roofline']['avg_launch_ms'], v['roofline']['k_parse_avg_ms'], v['roofline']['frac'], v['bitexact'])
PY
