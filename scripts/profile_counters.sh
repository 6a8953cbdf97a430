#!/bin/bash
# Collect PMC counters for the fused kernel, one rocprofv3 pass per counter group
# (counters only, no tracing domains).  Usage: scripts/profile_counters.sh OUTDIR [groups...]
# BENCH_ARGS: extra bench.py arguments (e.g. "--dataset syn_aids10knef --emulate-world 8").
set -u
OUT=${1:-gpurun_out/pmc}
shift || true
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/$OUT"
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > "$ROOT/$OUT/counters_list.txt" 2>&1 || true
GROUPS_DEFAULT=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_VALU_MFMA_BUSY_CYCLES"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_F32 GRBM_GUI_ACTIVE"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
if [ $# -gt 0 ]; then GROUPS_LIST=("$@"); else GROUPS_LIST=("${GROUPS_DEFAULT[@]}"); fi
i=0
for grp in "${GROUPS_LIST[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d "$ROOT/$OUT/pass$i" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --cpu-sample -1 ${BENCH_ARGS:-} > "$ROOT/$OUT/pass$i.log" 2>&1
  rc=$?
  echo "pass $i [$grp] rc=$rc" >> "$ROOT/$OUT/summary.txt"
  if [ $rc -ge 124 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
exit 0
