#!/bin/bash
# A/B of environment settings on the bench's headline configs (one gpurun call, one box):
#   ENVS="BNFLAC_DECODE_SYS=0;BNFLAC_DECODE_SYS=1" CFGS="C2 C3 C4 C5" ROUNDS=2 TAG=ab bash tools/ab_env.sh
# Each (round, env, cfg) runs bench.py without legs / baselines and prints the decode launch,
# k_parse and step times; the JSON lines go to gpurun_out/${TAG}_<cfg>_<i>_<round>.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-ab}
IFS=';' read -ra EV <<< "${ENVS:-BNFLAC_DECODE_SYS=0;BNFLAC_DECODE_SYS=1}"
for r in $(seq 1 ${ROUNDS:-1}); do
  for c in ${CFGS:-C2 C3 C4 C5}; do
    x=""; [ $c = C5 ] && x="--c5-batch"
    i=0
    for e in "${EV[@]}"; do
      out=gpurun_out/${TAG}_${c}_${i}_${r}.json
      env $e timeout -k 10 ${BENCH_TIMEOUT:-240} python3 bench.py --config $c $x --steps ${STEPS:-5} --warmup 2 --legs= \
          --no-cpu-baseline --no-pcie --no-index --no-reader ${EXTRA:-} --out $out > $out.log 2>&1
      rc=$?
      [ $rc -eq 0 ] || { echo "$c [$e] rc=$rc"; tail -5 $out.log; exit $rc; }
      python3 - "$out" "$c" "$e" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d["roofline"]
print(f"{sys.argv[2]} [{sys.argv[3]}] {d['value']:.1f} MS/s step {d['ms_per_step']:.3f} ms decode {r['avg_launch_ms']:.3f} ms "
      f"parse {r['k_parse_avg_ms']:.3f} ms frac {r['frac']:.3f} step_frac {r['step_frac']:.3f} bitexact {d['bitexact']}")
PY
      i=$((i + 1))
    done
  done
done
