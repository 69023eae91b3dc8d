set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread tests -m gpu -p no:cacheprovider > gpurun_out/r3g_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r3g_pytest.log
[ $rc -le 1 ] || exit $rc
AB_VAR=BNFLAC_ST_CRC_FIRST bash tools/ab_env.sh 0 1 2 3
