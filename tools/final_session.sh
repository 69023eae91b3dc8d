#!/bin/bash
# Round-end measurement session (one gpurun call): every GPU test, a rocprofv3 kernel trace
# + stats of each config's bench run, and the PMC passes (counters only, one rocprofv3 run
# per pass) that tools/pmc_summary.py turns into profiles/traffic_<cfg>_b<B>.json.
#   TAG=r4final bash tools/final_session.sh          (stage 1: tests + kernel traces)
#   TAG=r4final STAGE=2 bash tools/final_session.sh  (stage 2: PMC passes + the default bench line)
# C5 runs its real flow (bench.py --config C5: c5_job over 8 distinct files).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r4final}
mkdir -p gpurun_out
if [ "${STAGE:-1}" = 1 ]; then
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu \
    > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for c in ${CFGS:-C2 C3 C4 C5}; do
  TAG=$TAG CFG=$c STEPS=5 bash tools/prof_cfg.sh > gpurun_out/${TAG}_prof_$c.txt 2>&1 || { cat gpurun_out/${TAG}_prof_$c.txt; exit 1; }
  head -8 gpurun_out/${TAG}_prof_$c.txt
done
echo "stage 1 done"; exit 0
fi
for c in ${CFGS:-C2 C3 C4 C5}; do
  PMC_BENCH_ARGS="--config $c --steps 2 --warmup 1 --legs= --no-cpu-baseline --no-pcie --no-index --no-reader" \
  PMC_SETS='FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES' \
  TAG=${TAG}_$c bash tools/pmc_session.sh || exit $?
done
# PMC summaries (profiles/traffic_<cfg>_b<B>.json: bench.py's roofline.traffic for this build),
# then the default bench line (every leg, CPU baselines) with them in place
for cb in "C2 1024 1024" "C3 256 1024" "C4 256 4096" "C5 8 469"; do
  set -- $cb
  python3 tools/pmc_summary.py gpurun_out/pmc_${TAG}_$1 $1 $2 $3 $TAG > gpurun_out/traffic_${1,,}_b$2.json || exit 1
  cp gpurun_out/traffic_${1,,}_b$2.json profiles/
done
timeout -k 10 900 python bench.py --out gpurun_out/${TAG}_bench.json > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/${TAG}_bench.json
[ $rc -eq 0 ] || exit $rc
echo "final session done"
