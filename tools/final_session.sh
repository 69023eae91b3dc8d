#!/bin/bash
# Round-end measurement session: GPU tests, bench, rocprofv3 kernel stats, then PMC passes
# (counters only, one rocprofv3 run per pass).  usage: TAG=r1u bash tools/final_session.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-final}
export TAG
bash tools/gpu_session.sh || exit $?
PMC_SETS='FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES
TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE' \
  bash tools/pmc_session.sh
