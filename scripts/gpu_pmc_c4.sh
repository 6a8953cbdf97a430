#!/bin/bash
# Stall / instruction-cache counters of the capacity-32 kernel (C4, emulated W = 8 rank)
# and of the headline kernel (C2).  Usage: scripts/gpu_pmc_c4.sh TAG
set -u
TAG=${1:-pmc_c4}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_IFETCH GRBM_GUI_ACTIVE"
G2="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ"
G3="SQ_INSTS_BRANCH SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
G4="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
BENCH_ARGS="--dataset syn_aids10knef --emulate-world 8" bash "$ROOT/scripts/profile_counters.sh" "gpurun_out/$TAG/c4" "$G1" "$G2" "$G3" "$G4" || exit $?
cat "$ROOT/gpurun_out/$TAG/c4/summary.txt"
bash "$ROOT/scripts/profile_counters.sh" "gpurun_out/$TAG/c2" "$G1" "$G2" || exit $?
cat "$ROOT/gpurun_out/$TAG/c2/summary.txt"
