#!/bin/bash
# One bench configuration under rocprofv3: a kernel-trace pass and PMC passes (one per
# counter group, each its own run), outputs under gpurun_out/TAG/<name>/.  Usage:
#   scripts/gpu_prof_cfg.sh TAG NAME "bench args" [more NAME "args" pairs...]
# Summarise with: python scripts/pmc_summary.py gpurun_out/TAG/NAME KERNEL_SUBSTRING PAIRS
set -u
TAG=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd /tmp && export TMPDIR=/tmp
while [ $# -ge 2 ]; do
  NAME=$1; ARGS=$2; shift 2
  OUT=$ROOT/gpurun_out/$TAG/$NAME
  mkdir -p "$OUT"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" $ARGS --cpu-sample -1 --json-out "$OUT/bench.json" > "$OUT/trace.log" 2>&1
  rc=$?; echo "$NAME trace rc=$rc" | tee -a "$ROOT/gpurun_out/$TAG/summary.txt"
  [ $rc -eq 0 ] || exit $rc
  i=0
  for grp in \
      "SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_MFMA_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH GRBM_GUI_ACTIVE" \
      "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $grp -d "$OUT/pass$i" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" $ARGS --steps 3 --warmup 1 --cpu-sample -1 > "$OUT/pass$i.log" 2>&1
    rc=$?; echo "$NAME pmc$i rc=$rc" | tee -a "$ROOT/gpurun_out/$TAG/summary.txt"
    [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
