#!/bin/bash
# A/B on the GPU: parity tests on the default library, then one bench line per
# library variant.  Usage: scripts/gpu_ab.sh TAG lib1.so [lib2.so ...]
set -u
TAG=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -m pytest tests -q -x -m gpu > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; tail -3 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
for lib in "$@"; do
  n=$(basename "$lib" .so)
  SG_LIB=$ROOT/$lib timeout -k 10 300 python bench.py --cpu-sample -1 --json-out "$OUT/bench_$n.json" > "$OUT/bench_$n.log" 2>&1
  rc=$?; echo "bench $n rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('$OUT/bench_$n.json'));print('$n', round(d['value']/1e6,1),'M pairs/s', round(d['ms_per_step'],3),'ms/step')"
done
