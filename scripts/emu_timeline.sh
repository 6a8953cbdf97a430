#!/bin/bash
# Emulated W-rank step timeline: bench line of one rank's share of a
# W-GPU step and its rocprof kernel trace.  Usage: scripts/emu_timeline.sh TAG [W]
# then: python scripts/step_timeline.py gpurun_out/TAG/trace/run_kernel_trace.csv
set -u
TAG=${1:-emu}
W=${2:-8}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 120 python bench.py --emulate-world $W --steps 200 --warmup 20 --cpu-sample -1 \
  --json-out "$OUT/emu$W.json" > "$OUT/emu$W.log" 2>&1
rc=$?; echo "emu$W rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --emulate-world $W --steps 50 --warmup 5 --cpu-sample -1 > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; exit $rc
