#!/bin/bash
# round 5, first GPU session: the VALU-mix microbench, the GPU suite, a short bench
mkdir -p gpurun_out
timeout -k 10 120 tools/ubench_mix > gpurun_out/ubench_mix.txt 2>&1; echo "ubench rc=$?"
TAG=r5a bash tools/gpu_quick.sh
