#!/bin/bash
# Round-6 A/B of the NTN weight-gradient kernel (Average / Attention stacks): the product
# library against ab/ variants, then one kernel trace per variant of the Average stack.
set -u
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-r06_f}
VARIANTS=${VARIANTS:-} MODES="avg att" NO_ROUND3=1 bash "$ROOT/scripts/gpu_round5.sh" "$TAG" skip || exit $?
cd /tmp && export TMPDIR=/tmp
OUT=$ROOT/gpurun_out/$TAG
for v in prod ${VARIANTS:-}; do
  n=$(basename "$v" .so)
  if [ "$v" = prod ]; then L=""; else L="$ROOT/$v"; fi
  SG_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$n" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --stack average --steps 20 --warmup 5 --cpu-sample -1 > "$OUT/trace_$n.log" 2>&1
  rc=$?; echo "trace $n rc=$rc" | tee -a "$OUT/summary.txt"
  [ $rc -eq 0 ] || exit $rc
done
