#!/bin/bash
# A/B of the product library against ab/ variants (scripts/gpu_round5.sh modes), then one
# kernel trace per library of the bench arguments TRACE_ARGS.  Usage:
#   VARIANTS="ab/x.so" MODES="c4" TRACE_ARGS="--dataset syn_aids10knef --steps 2 --warmup 1" \
#     scripts/gpu_r6_ab_trace.sh TAG
set -u
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-r06_x}
NO_ROUND3=1 bash "$ROOT/scripts/gpu_round5.sh" "$TAG" skip || exit $?
cd /tmp && export TMPDIR=/tmp
OUT=$ROOT/gpurun_out/$TAG
for v in prod ${VARIANTS:-}; do
  n=$(basename "$v" .so)
  if [ "$v" = prod ]; then L=""; else L="$ROOT/$v"; fi
  SG_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$n" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" $TRACE_ARGS --cpu-sample -1 > "$OUT/trace_$n.log" 2>&1
  rc=$?; echo "trace $n rc=$rc" | tee -a "$OUT/summary.txt"
  [ $rc -eq 0 ] || exit $rc
done
