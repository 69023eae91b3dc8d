set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3n_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r3n_tests.log; exit 1; }
tail -2 gpurun_out/r3n_tests.log
for v in dwfwd dwrev; do cp ab/$v.so birdnest/audio_amd/lib/libbnflac.so
for m in 0 2; do for c in C2 C5; do
  [ $v = dwfwd ] && [ $m = 0 ] && continue
  extra=""; [ $c = C5 ] && extra="--c5-batch"
  BNFLAC_DECODE_WAVE=$m timeout -k 10 300 python bench.py --config $c $extra --batches 1 --steps 10 --warmup 2 --legs= --no-cpu-baseline --no-pcie --no-index --out gpurun_out/r3n_${c}_${v}_m$m.json > gpurun_out/r3n_${c}_m$m.log 2>&1 || { echo "bench $c $m failed"; tail gpurun_out/r3n_${c}_m$m.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r3n_${c}_${v}_m$m.json')); r=d['roofline']
print('$v $c mode $m', 'decode_ms', r['avg_launch_ms'], 'parse_ms', r['k_parse_avg_ms'], 'step_ms', d['ms_per_step'], 'bitexact', d['bitexact'], 'reader', d.get('reader',{}).get('value'), d.get('reader',{}).get('from_c'))"
done; done; done
cp ab/dwrev.so birdnest/audio_amd/lib/libbnflac.so
