set -u
mkdir -p gpurun_out
timeout -k 10 60 ./tools/ubench_mad > gpurun_out/r3a_ubench_mad.txt 2>&1; echo "ubench rc=$?"; cat gpurun_out/r3a_ubench_mad.txt
timeout -k 10 900 python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread tests -m gpu -p no:cacheprovider > gpurun_out/r3a_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/r3a_pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pcie --out gpurun_out/r3a_bench.json > gpurun_out/r3a_bench.log 2>&1; echo "bench rc=$?"; tail -2 gpurun_out/r3a_bench.log | cut -c1-600
