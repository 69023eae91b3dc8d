#!/bin/bash
# round 5: PMC passes on C2 (B = 256) for the round-5 k_decode_st
export PMC_BENCH_ARGS="--batches 256 --steps 2 --warmup 1 --legs= --no-cpu-baseline --no-pcie --no-index --no-reader"
export PMC_SETS='SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES
SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT
FETCH_SIZE
WRITE_SIZE'
TAG=r5g bash tools/pmc_session.sh && python3 tools/pmc_kernel.py gpurun_out/pmc_r5g k_decode_st k_parse
