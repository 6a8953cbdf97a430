#!/bin/bash
# One GPU session: GPU tests, bench (with CPU baseline), rocprof kernel-trace
# stats and PMC HBM-traffic passes for the same bench command.
# Usage: scripts/gpu_round.sh TAG   (outputs under gpurun_out/TAG)
set -u
TAG=${1:-run}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -m pytest tests -q -m gpu > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest_gpu rc=$rc" | tee -a "$OUT/summary.txt"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc" | tee -a "$OUT/summary.txt"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --json-out "$OUT/bench.json" > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc" | tee -a "$OUT/summary.txt"
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 10 --warmup 2 --cpu-sample -1 > "$OUT/trace.log" 2>&1
rc=$?; echo "rocprof trace rc=$rc" | tee -a "$OUT/summary.txt"
[ $rc -eq 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d "$OUT/pmc_$c" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --cpu-sample -1 > "$OUT/pmc_$c.log" 2>&1
  rc=$?; echo "pmc $c rc=$rc" | tee -a "$OUT/summary.txt"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
