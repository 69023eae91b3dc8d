#!/bin/bash
# round 5: instruction-class microbench (second set) and the C5 parse A/B
mkdir -p gpurun_out
timeout -k 10 120 tools/ubench_mix2 > gpurun_out/ubench_mix2.txt 2>&1; echo "ubench2 rc=$?"
timeout -k 10 300 python tools/c5_parse_ab.py > gpurun_out/c5ab.txt 2>&1; echo "c5ab rc=$?"; cat gpurun_out/c5ab.txt
BNFLAC_PW_STATS=1 timeout -k 10 300 python tools/c5_parse_ab.py > gpurun_out/c5ab_stats.txt 2>&1; echo "c5ab stats rc=$?"; cat gpurun_out/c5ab_stats.txt
