#!/bin/bash
# C5 kernel breakdown with the chunk pipeline off (SG_WEB_PIPE=0: kernel-trace durations do
# not overlap), then PMC passes over the same step: issue/wait counters and HBM fetch.
# Usage: scripts/gpu_c5_prof3.sh TAG
set -u
TAG=${1:-c5prof3}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export SG_WEB_PIPE=0
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --dataset syn_web --steps 1 --warmup 1 --cpu-sample -1 > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 400 rocprofv3 --pmc $grp -d "$OUT/pmc$i" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --dataset syn_web --steps 1 --warmup 1 --cpu-sample -1 > "$OUT/pmc$i.log" 2>&1
  rc=$?; echo "pmc$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
