set -u
mkdir -p gpurun_out
for c in "C2 1" "C2 4" "C2 16" "C3 1" "C3 8" "C5 1" "C4 1"; do timeout -k 10 120 python tools/pw_stats.py $c 2>&1 | grep "mode" | head -2; done
