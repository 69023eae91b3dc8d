#!/bin/bash
# One gpurun session: GPU parity tests -> bench -> rocprofv3 kernel trace of the bench.
# Every GPU step has its own time limit; a crash/timeout (not a plain test failure)
# stops the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
TAG=${TAG:-r1}
STEPS=${STEPS:-tests,bench,prof}
export PYTHONUNBUFFERED=1
stop() { echo "STOP: $1 rc=$2"; exit "$2"; }
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -q --maxfail=30 -p no:cacheprovider ${PYTEST_ARGS:-} > "$OUT/pytest_gpu_$TAG.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu_$TAG.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then stop pytest $rc; fi
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:-} --out "$OUT/bench_$TAG.json" > "$OUT/bench_$TAG.log" 2>&1
  rc=$?; echo "bench rc=$rc"; tail -3 "$OUT/bench_$TAG.log"
  [ $rc -eq 0 ] || stop bench $rc
fi
if [[ $STEPS == *prof* ]]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 ${PROF_TIMEOUT:-600} rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" ${PROF_ARGS:---steps 5 --warmup 1 --no-cpu-baseline --no-pcie --no-index --no-reader} > "$OUT/prof_$TAG.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 "$OUT/prof_$TAG.log"
  [ $rc -eq 0 ] || stop rocprof $rc
fi
echo "session done"
