#!/bin/bash
# Fixed-cost diagnostics for strong scaling: per-wave timeline of the
# fused kernel at W = 1 and 8 (timing build), the emulated W = 8 rank's bench line and
# its per-step kernel timeline.  Build the timing library first:
#   python graphembedding_amd/build.py --out graphembedding_amd/lib/libsiamese_timing.so -DSG_FAST_TIMING=1
# Usage: scripts/scaling_diag.sh TAG ; then python scripts/step_timeline.py gpurun_out/TAG/trace8/run_kernel_trace.csv
set -eu
TAG=${1:-diag}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
SG_LIB=graphembedding_amd/lib/libsiamese_timing.so timeout -k 10 120 python scripts/fast_timing.py 1 8 > "$OUT/timing.log" 2>&1
timeout -k 10 120 python bench.py --emulate-world 8 --steps 200 --warmup 20 --cpu-sample -1 > "$OUT/emu8.log" 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d "$OUT/trace8" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --emulate-world 8 --steps 50 --warmup 5 --cpu-sample -1 > "$OUT/trace8.log" 2>&1
