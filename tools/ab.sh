#!/bin/bash
# A/B timing of library variants on one box: ab/<name>.so copied over the in-tree library
# before each bench run.  usage: [AB_ROUNDS=2] tools/ab.sh name1 name2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LIB=birdnest/audio_amd/lib/libbnflac.so
cp "$LIB" ab/_orig.so
for r in $(seq 1 ${AB_ROUNDS:-2}); do
  for v in "$@"; do
    cp "ab/$v.so" "$LIB"
    timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pcie --no-index ${AB_ARGS:-} > "gpurun_out/ab_${v}_$r.json" 2>/dev/null || { echo "bench $v failed"; cp ab/_orig.so "$LIB"; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/ab_${v}_$r.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$v', 'round $r', 'value', d['value'], 'k_decode_ms', r['avg_launch_ms'], 'k_parse_ms', r['k_parse_avg_ms'], 'bitexact', d['bitexact'])"
  done
done
cp ab/_orig.so "$LIB"
