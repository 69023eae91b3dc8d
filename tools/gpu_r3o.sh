set -u
mkdir -p gpurun_out
for c in C2 C5; do
  extra=""; [ $c = C5 ] && extra="--c5-batch"
  timeout -k 10 300 python bench.py --config $c $extra --batches 1 --steps 5 --warmup 1 --legs= --no-cpu-baseline --no-pcie --no-index --no-reader --stats --out gpurun_out/r3o_${c}.json > gpurun_out/r3o_${c}.log 2>&1 || { echo "bench $c failed"; tail gpurun_out/r3o_${c}.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r3o_${c}.json')); r=d['roofline']
print('$c', 'decode_ms', r['avg_launch_ms'], d.get('stats'))"
done
