#!/bin/bash
# C2 decode-read attribution (one box, counters only): FETCH_SIZE of the decode and parse
# kernels with the CRC-16 hand-off off (BNFLAC_CRC_MODE=0: the tail re-reads whole frames),
# on (mode 1, the default: the tail re-reads channel 1), and with the CRC skipped
# (BNFLAC_ABLATE=1: the ring DMAs alone).  Output: gpurun_out/pmc_abl_<variant>/...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
ARGS="--steps 2 --warmup 1 --legs= --no-cpu-baseline --no-pcie --no-index --no-reader"
cd /tmp && export TMPDIR=/tmp
run() { # name, env assignment, counters
  local out=$ROOT/gpurun_out/pmc_abl_$1
  mkdir -p "$out"
  env_kv=$2
  export $env_kv
  timeout -k 10 300 rocprofv3 --pmc $3 -d "$out" -o run --output-format csv -- python3 "$ROOT/bench.py" $ARGS > "$out.log" 2>&1
  local rc=$?
  unset ${env_kv%%=*}
  echo "$1 ($3) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$out.log"; exit $rc; }
}
run mode0 BNFLAC_CRC_MODE=0 FETCH_SIZE
run mode1 BNFLAC_CRC_MODE=1 FETCH_SIZE
run nocrc BNFLAC_ABLATE=1 FETCH_SIZE
run write1 BNFLAC_CRC_MODE=1 WRITE_SIZE
echo "pmc ablate done"
