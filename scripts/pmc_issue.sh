#!/bin/bash
# Issue-pressure counters for the fused kernel: scripts/pmc_issue.sh OUTTAG [lib.so]
set -u
TAG=$1; LIB=${2:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
[ -n "$LIB" ] && export SG_LIB=$ROOT/$LIB
bash "$ROOT/scripts/profile_counters.sh" "gpurun_out/$TAG" \
  "SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAVES"
