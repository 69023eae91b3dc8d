#!/bin/bash
# round 5: offset-form ring DMAs, packed 16-bit decorrelation, bulk parse steps (k <= 9) --
# parity suite, the C2-C4 bench legs, then C3's store / CRC ablation
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r5m_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r5m_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-pcie --no-reader --no-index --legs C3,C4 --out gpurun_out/r5m_bench.json > gpurun_out/r5m_bench.log 2>&1; rc=$?; echo "bench rc=$rc"
[ $rc -eq 0 ] || exit $rc
python - <<PY
import json
d=json.loads(open('gpurun_out/r5m_bench.json').read())
print('C2', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['k_parse_avg_ms'], d['roofline']['frac'], d['bitexact'])
for k,v in d.get('legs',{}).items(): print(k, v['value'], v['roofline']['avg_launch_ms'], v['roofline']['k_parse_avg_ms'], v['roofline']['frac'], v['bitexact'])
PY
ENVS="BNFLAC_ABLATE=0;BNFLAC_ABLATE=1;BNFLAC_ABLATE=2" CFGS="C3" ROUNDS=1 TAG=abl5c3 bash tools/ab_env.sh
