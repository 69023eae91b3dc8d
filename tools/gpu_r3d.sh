set -u
mkdir -p gpurun_out
for seg in ${SEGS:-8 4}; do
BNFLAC_PW_SEG=$seg timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_parse_wave.py -p no:cacheprovider > gpurun_out/r3d_pw_$seg.log 2>&1; rc=$?; echo "seg $seg parse_wave tests rc=$rc"; tail -3 gpurun_out/r3d_pw_$seg.log
[ $rc -le 1 ] || exit $rc
BNFLAC_PW_SEG=$seg timeout -k 10 300 python tools/pw_stats.py C5 8 2>&1 | tail -4
BNFLAC_PW_SEG=$seg BNFLAC_PW_STATS=1 timeout -k 10 300 python tools/pw_stats.py C5 8 2>&1 | tail -2 | head -1
BNFLAC_PW_SEG=$seg timeout -k 10 300 python tools/pw_stats.py C2 64 2>&1 | tail -4
done
