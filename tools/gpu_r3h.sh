set -u
mkdir -p gpurun_out
for r in 1 2; do for v in fwd rev; do cp ab/$v.so birdnest/audio_amd/lib/libbnflac.so
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-pcie --no-index --no-reader --legs=C3,C4,C5 --out gpurun_out/ab_pred_${v}_$r.json > /dev/null 2>&1 || { echo fail; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ab_pred_${v}_$r.json'))
print('$v', [(k, v['roofline']['avg_launch_ms'], v['roofline']['k_parse_avg_ms'], v['bitexact']) for k,v in d['legs'].items()])"
done; done
cp ab/rev.so birdnest/audio_amd/lib/libbnflac.so
