#!/bin/bash
# A/B timing of one library under environment settings: usage AB_VAR=NAME tools/ab_env.sh v1 v2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in $(seq 1 ${AB_ROUNDS:-2}); do
  for v in "$@"; do
    env ${AB_VAR}=$v timeout -k 10 200 python bench.py --steps ${AB_STEPS:-10} --warmup 2 --no-cpu-baseline --no-pcie --no-index --no-reader --legs= ${AB_ARGS:-} > "gpurun_out/abenv_${AB_VAR}_${v}_$r.json" 2>/dev/null || { echo "bench $v failed"; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/abenv_${AB_VAR}_${v}_$r.json').read().strip().splitlines()[-1]);r=d['roofline'];print('${AB_VAR}=$v', 'round $r', 'value', d['value'], 'k_decode_ms', r['avg_launch_ms'], 'k_parse_ms', r['k_parse_avg_ms'], 'bitexact', d['bitexact'])"
  done
done
