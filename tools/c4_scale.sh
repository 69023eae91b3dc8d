set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/c4scale.txt; : > $O
for b in 1 8 32 64 128 256; do
  timeout -k 10 240 python bench.py --config C4 --batches $b --steps 3 --warmup 1 --legs '' --no-cpu-baseline --no-pcie --no-index --no-reader > gpurun_out/c4s_$b.json 2>gpurun_out/c4s_$b.err || { echo "fail $b" >> $O; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/c4s_$b.json').read().strip().splitlines()[-1]); r=d['roofline']; print('B=$b', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['k_parse_avg_ms'])" >> $O
done
for b in 32 256; do
  BNFLAC_DECODE_SYS=1 timeout -k 10 240 python bench.py --config C4 --batches $b --steps 3 --warmup 1 --legs '' --no-cpu-baseline --no-pcie --no-index --no-reader > gpurun_out/c4sys_$b.json 2>gpurun_out/c4sys_$b.err || { echo "fail sys $b" >> $O; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/c4sys_$b.json').read().strip().splitlines()[-1]); r=d['roofline']; print('SYS B=$b', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['k_parse_avg_ms'])" >> $O
done
cat $O
