#!/bin/bash
# A/B of library variants ab/<name>.so on one box, C2 headline + optional legs; optional env
# per variant as name:ENV=VAL.  usage: AB_ROUNDS=2 AB_ARGS="--legs=C4" bash tools/ab2.sh v0 v2 v2:BNFLAC_DECODE_SERIAL=1
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LIB=birdnest/audio_amd/lib/libbnflac.so
cp "$LIB" ab/_orig.so
for r in $(seq 1 ${AB_ROUNDS:-2}); do
  for spec in "$@"; do
    v=${spec%%:*}; ev=""; [ "$spec" != "$v" ] && ev=${spec#*:}
    cp "ab/$v.so" "$LIB"
    tag=$(echo "$spec" | tr ':=' '__')
    env $ev timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pcie --no-index --no-reader ${AB_ARGS:-} \
        --out "gpurun_out/ab_${tag}_$r.json" > "gpurun_out/ab_${tag}_$r.log" 2>&1 || { echo "bench $spec failed"; tail -5 "gpurun_out/ab_${tag}_$r.log"; cp ab/_orig.so "$LIB"; exit 1; }
    python3 - "gpurun_out/ab_${tag}_$r.json" "$spec" "$r" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d["roofline"]
s = f"{sys.argv[2]:36s} r{sys.argv[3]} C2 {d['value']:.0f} dec {r['avg_launch_ms']:.3f} parse {r['k_parse_avg_ms']:.3f} ok {d['bitexact']}"
for k, v in d.get("legs", {}).items():
    s += f" | {k} {v['value']:.0f} dec {v['roofline']['avg_launch_ms']:.3f} parse {v['roofline']['k_parse_avg_ms']:.3f} ok {v['bitexact']}"
print(s)
PY
  done
done
cp ab/_orig.so "$LIB"
