set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3i_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r3i_tests.log; exit 1; }
tail -3 gpurun_out/r3i_tests.log
AB_ROUNDS=2 AB_ARGS="--legs= --no-reader" bash tools/ab.sh pair tail2 tail4 tail8
