#!/bin/bash
# rocprofv3 kernel trace + stats of one bench config (headline only, no side legs).
# usage: TAG=r2x CFG=C4 bash tools/prof_cfg.sh  -> gpurun_out/prof_${TAG}_${CFG}/
set -u
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_${TAG:-x}_${CFG:-C4}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 ${PROF_TIMEOUT:-300} rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --config ${CFG:-C4} --steps ${STEPS:-5} --warmup 1 --legs= --no-cpu-baseline --no-pcie \
    --no-index --no-reader ${EXTRA:-} > "$OUT.log" 2>&1
rc=$?; echo "prof $CFG rc=$rc"
[ $rc -eq 0 ] || { tail -5 "$OUT.log"; exit $rc; }
python3 - "$OUT/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:50]:50s} calls {r['Calls']:>5s} avg_ms {float(r['AverageNs'])/1e6:9.4f} total_ms {float(r['TotalDurationNs'])/1e6:9.3f}")
PY
