# A/B of the CRC-16 hand-off modes (BNFLAC_CRC_MODE 0 / 1 / 2, bnflac_kernels.hip crc_mode) on
# C2 + C3, after the GPU suite: one gpurun call, e.g.  gpurun -- 'bash tools/crc_mode_ab.sh r6m'
set -o pipefail
TAG=${1:-crc}
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/crc_handoff_check.py --copies 128 > gpurun_out/${TAG}_chk.log 2>&1 || exit $?
tail -3 gpurun_out/${TAG}_chk.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo pytest rc=$rc
tail -3 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for m in 1 0 2 1 0 2; do
  BNFLAC_CRC_MODE=$m timeout -k 10 300 python bench.py --steps 10 --warmup 2 --legs=C3 --no-cpu-baseline --no-pcie --no-reader --no-index --out gpurun_out/${TAG}_m$m.json > gpurun_out/${TAG}_m$m.log 2>&1 || { echo bench fail; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_m$m.json')); r=d['roofline']
print('mode $m C2', d['value'], r['avg_launch_ms'], r['k_parse_avg_ms'], r['frac'], d['bitexact'], d['ms_per_step'])
for k,v in d.get('legs',{}).items(): print('   ', k, v['value'], v['roofline']['avg_launch_ms'], v['roofline']['k_parse_avg_ms'], v['bitexact'], v['ms_per_step'])"
done
