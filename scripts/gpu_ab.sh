#!/bin/bash
# A/B on the GPU: parity tests on the default library, then one bench line per
# library variant.  Usage: scripts/gpu_ab.sh TAG lib1.so [lib2.so ...]
set -u
TAG=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -m pytest ${TESTS:-tests} -q -x -m gpu > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; tail -3 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
# REPS rounds over the variants (alternating), 100 timed steps each
# (BENCH_ARGS: extra bench.py flags, TESTS: pytest targets)
REPS=${REPS:-2}
for rep in $(seq 1 $REPS); do
  for lib in "$@"; do
    n=$(basename "$lib" .so)
    SG_LIB=$ROOT/$lib timeout -k 10 300 python bench.py --cpu-sample -1 --steps 100 --warmup 10 ${BENCH_ARGS:-} \
      --json-out "$OUT/bench_${n}_$rep.json" > "$OUT/bench_${n}_$rep.log" 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "bench $n rc=$rc"; exit $rc; }
    python -c "import json;d=json.load(open('$OUT/bench_${n}_$rep.json'));print('$n rep $rep', round(d['value']/1e6,1),'M pairs/s', round(d['ms_per_step'],4),'ms/step')"
  done
done
