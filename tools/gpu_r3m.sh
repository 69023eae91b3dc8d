set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3m_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r3m_tests.log; exit 1; }
tail -2 gpurun_out/r3m_tests.log
run() { # name lib env...
  local v=$1 lib=$2; shift 2
  cp ab/$lib.so birdnest/audio_amd/lib/libbnflac.so
  env "$@" timeout -k 10 300 python bench.py --config C3 --steps 5 --warmup 1 --no-cpu-baseline --no-pcie --no-index --no-reader --legs=C5,C4 --out gpurun_out/r3m_${v}.json > /dev/null 2>&1 || { echo fail $v; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r3m_${v}.json'))
print('$v', 'C3', d['roofline']['avg_launch_ms'], d['bitexact'], [(k, v['roofline']['avg_launch_ms'], v['bitexact']) for k,v in d['legs'].items()])"
}
for r in 1 2; do
run base$r base X=1
run pre$r pre X=1
done
cp ab/pre.so birdnest/audio_amd/lib/libbnflac.so
