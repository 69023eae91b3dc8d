# LDS counters of the C2 decode with and without the CRC-16 tail (BNFLAC_ABLATE=1)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/r3j_counters.txt 2>&1 || true
cd $GRAFT_REPO_ROOT
export PMC_BENCH_ARGS="--steps 2 --warmup 1 --legs= --no-cpu-baseline --no-pcie --no-index --no-reader"
export PMC_SETS="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
export PMC_TIMEOUT=120
TAG=r3j_crc bash tools/pmc_session.sh || exit 1
BNFLAC_ABLATE=1 TAG=r3j_nocrc bash tools/pmc_session.sh || exit 1
for c in C5 C3; do
timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --legs= --no-cpu-baseline --no-pcie --no-index --no-reader --stats --ablate 1,2,4,8,12 --out gpurun_out/r3j_abl_$c.json > /dev/null 2>&1 || { echo "abl $c failed"; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r3j_abl_$c.json')); print('$c', d['value'], d['roofline']['avg_launch_ms'], d.get('stats'), d.get('ablation'))"
done
