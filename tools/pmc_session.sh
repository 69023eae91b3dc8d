#!/bin/bash
# PMC counter passes over a short bench run (one rocprofv3 invocation per pass; counters
# only, no trace domains).  Output: gpurun_out/pmc_$TAG/<pass>/...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_${TAG:-r1}
mkdir -p "$OUT"
ARGS=${PMC_BENCH_ARGS:---steps 2 --warmup 1 --no-cpu-baseline --no-pcie --no-index --no-reader}
cd /tmp && export TMPDIR=/tmp
i=0
while IFS= read -r ctrs; do
  [ -z "$ctrs" ] && continue
  i=$((i+1))
  timeout -k 10 ${PMC_TIMEOUT:-300} rocprofv3 --pmc $ctrs -d "$OUT/p$i" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i ($ctrs) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$OUT/p$i.log"; exit $rc; }
done <<< "${PMC_SETS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES
FETCH_SIZE
WRITE_SIZE
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT}"
echo "pmc done"
