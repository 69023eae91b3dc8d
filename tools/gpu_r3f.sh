set -u
mkdir -p gpurun_out
[ "${SKIPTEST:-0}" = 1 ] || timeout -k 10 900 python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread tests -m gpu -p no:cacheprovider > gpurun_out/r3f_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/r3f_pytest.log
[ $rc -le 1 ] || exit $rc
AB_ROUNDS=2 AB_ARGS="--legs= --no-reader" bash tools/ab.sh single pair
