#!/bin/bash
# C5 (Web) GPU session: bench line + rocprof kernel stats.  Usage: scripts/web_round.sh TAG [bench args]
set -u
TAG=${1:-web}; shift || true
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python bench.py --dataset syn_web "$@" --json-out "$OUT/bench.json" > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 "$OUT/bench.log"
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --dataset syn_web --steps 1 --warmup 1 --cpu-sample -1 > "$OUT/trace.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
exit $rc
