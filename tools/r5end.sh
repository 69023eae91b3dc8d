#!/bin/bash
# round 5 end: the committed tree as the driver runs it -- GPU tests, smoke(), a short default bench
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r5end_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r5end_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5end_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r5end_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --legs= --out gpurun_out/r5end_bench.json > gpurun_out/r5end_bench.log 2>&1; rc=$?; echo "bench rc=$rc"
python3 -c "
import json; d=json.load(open('gpurun_out/r5end_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['roofline'].get('traffic'), d['bitexact'], d['kernels_sha'])"
