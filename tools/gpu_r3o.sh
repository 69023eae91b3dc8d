set -u
mkdir -p gpurun_out
cp ab/ow.so birdnest/audio_amd/lib/libbnflac.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode_wave.py tests/test_gpu_parse_wave.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3o_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r3o_tests.log; exit 1; }
tail -2 gpurun_out/r3o_tests.log
for v in timers owtimers noow ow; do cp ab/$v.so birdnest/audio_amd/lib/libbnflac.so
for c in C2 C5; do
  extra=""; [ $c = C5 ] && extra="--c5-batch"
  BNFLAC_DECODE_WAVE=1 timeout -k 10 300 python bench.py --config $c $extra --batches 1 --steps 5 --warmup 1 --legs= --no-cpu-baseline --no-pcie --no-index --no-reader --stats --out gpurun_out/r3o_${c}_$v.json > gpurun_out/r3o_${c}.log 2>&1 || { echo "bench $c failed"; tail gpurun_out/r3o_${c}.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r3o_${c}_$v.json')); r=d['roofline']
print('$v $c', 'decode_ms', r['avg_launch_ms'], 'parse_ms', r['k_parse_avg_ms'], d['bitexact'], d.get('stats',{}).get('cycles_per_wave'))"
done; done
cp ab/ow.so birdnest/audio_amd/lib/libbnflac.so
