# C5 (batch) ablations + stats, and the WRITE_SIZE calibration of the store micro-benchmark
set -u
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config C5 --c5-batch --steps 5 --warmup 1 --legs= --no-cpu-baseline --no-pcie --no-index --no-reader --stats --ablate 1,2,4,8,12 --out gpurun_out/r3l_abl_C5.json > gpurun_out/r3l_abl_C5.log 2>&1 || { echo "abl C5 failed"; tail gpurun_out/r3l_abl_C5.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r3l_abl_C5.json')); print('C5', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['k_parse_avg_ms'], d.get('stats'), d.get('ablation'))"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $ROOT/gpurun_out/r3l_store -o run --output-format csv -- $ROOT/tools/ubench_store > $ROOT/gpurun_out/r3l_store.log 2>&1 || { echo "store pmc failed"; tail $ROOT/gpurun_out/r3l_store.log; exit 1; }
cat $ROOT/gpurun_out/r3l_store.log | grep run=
python3 -c "
import csv,glob
for f in glob.glob('$ROOT/gpurun_out/r3l_store/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)): print(r['Kernel_Name'][:40], r['Counter_Name'], r['Counter_Value'])"
