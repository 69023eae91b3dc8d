#!/bin/bash
# the round-end driver's steps on this tree: smoke() and a short default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pcie --no-reader --no-index --out gpurun_out/final_check.json > gpurun_out/final_check.log 2>&1; echo "bench rc=$?"
python3 -c "
import json; d=json.loads(open('gpurun_out/final_check.json').read().strip().split(chr(10))[-1])
print('C2', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['bitexact'])
[print(k, v['value'], v['roofline']['avg_launch_ms'], v['bitexact']) for k, v in d.get('legs', {}).items()]"
