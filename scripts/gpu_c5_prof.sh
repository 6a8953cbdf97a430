#!/bin/bash
# C5 kernel breakdown: rocprofv3 kernel trace of one C5 step, then PMC wait/issue counters
# of the instance kernels (each pass its own run).  Usage: scripts/gpu_c5_prof.sh TAG
set -u
TAG=${1:-c5prof}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --dataset syn_web --steps 1 --warmup 1 --cpu-sample -1 > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 400 rocprofv3 --pmc $grp -d "$OUT/pmc$i" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --dataset syn_web --steps 1 --warmup 1 --cpu-sample -1 > "$OUT/pmc$i.log" 2>&1
  rc=$?; echo "pmc$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
