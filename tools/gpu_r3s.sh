#!/bin/bash
# C3 counters of k_decode_sw (one PMC pass) and a kernel trace with stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r3s_c3 PMC_BENCH_ARGS="--config C3 --legs= --steps 2 --warmup 1 --no-cpu-baseline --no-pcie --no-index --no-reader" \
PMC_SETS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" bash tools/pmc_session.sh || exit 1
ROOT=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/r3s_prof -o run --output-format csv -- python3 $ROOT/bench.py --config C3 --legs= --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --no-index --no-reader > $ROOT/gpurun_out/r3s_prof.log 2>&1; echo "prof rc=$?"
find $ROOT/gpurun_out/r3s_prof -name "*kernel_stats.csv" -exec head -12 {} \;
find $ROOT/gpurun_out/pmc_r3s_c3 -name "*counter_collection.csv" | head -2
