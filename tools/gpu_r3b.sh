set -u
mkdir -p gpurun_out
T=${TAG:-r3c}
timeout -k 10 300 python -u -m pytest -q --maxfail=5 --timeout 120 --timeout-method thread tests/test_gpu_parse_wave.py -p no:cacheprovider > gpurun_out/${T}_pw.log 2>&1; rc=$?; echo "parse_wave rc=$rc"; tail -30 gpurun_out/${T}_pw.log
[ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread tests -m gpu -p no:cacheprovider > gpurun_out/${T}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/${T}_pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu-baseline --out gpurun_out/${T}_c5.json > gpurun_out/${T}_c5.log 2>&1; echo "c5 rc=$?"
BNFLAC_PARSE_WAVE=0 timeout -k 10 300 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu-baseline --out gpurun_out/${T}_c5_lane.json > gpurun_out/${T}_c5_lane.log 2>&1; echo "c5 lane rc=$?"
BNFLAC_PARSE_WAVE=1 timeout -k 10 300 python bench.py --steps 5 --warmup 1 --legs '' --no-cpu-baseline --no-pcie --no-index --no-reader --out gpurun_out/${T}_c2_wave.json > gpurun_out/${T}_c2_wave.log 2>&1; echo "c2 wave rc=$?"
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --legs '' --no-cpu-baseline --no-pcie --out gpurun_out/${T}_c2.json > gpurun_out/${T}_c2.log 2>&1; echo "c2 rc=$?"
python - <<PY
import json
for f in ['${T}_c5','${T}_c5_lane','${T}_c2_wave','${T}_c2']:
    try:
        d=json.loads(open('gpurun_out/'+f+'.json').read())
        r=d['roofline']; print(f, d['value'], 'step', d['ms_per_step'], 'dec', r['avg_launch_ms'], 'parse', r['k_parse_avg_ms'], 'frac', r['frac'], 'stepfrac', r['step_frac'], d['bitexact'], d.get('reader',{}).get('from_c'), d.get('indexer',{}).get('ms'))
    except Exception as e: print(f, 'ERR', e)
PY
