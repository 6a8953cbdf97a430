#!/bin/bash
# Quick GPU check: parity tests, then one bench line.  Usage: scripts/gpu_quick.sh TAG [pytest -k expr]
set -u
TAG=${1:-quick}
K=${2:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
if [ -n "$K" ]; then
  timeout -k 10 600 python -m pytest tests -q -x -m gpu -k "$K" > "$OUT/pytest_gpu.log" 2>&1
else
  timeout -k 10 600 python -m pytest tests -q -x -m gpu > "$OUT/pytest_gpu.log" 2>&1
fi
rc=$?; echo "pytest_gpu rc=$rc"; tail -3 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --cpu-sample -1 --json-out "$OUT/bench.json" > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"
exit $rc
