#!/bin/bash
# Timing-only A/B (no parity tests: for throwaway ablation builds whose results are
# not meant to be right).  Usage: scripts/gpu_bench_variants.sh TAG lib1.so [lib2.so ...]
# REPS rounds over the variants (alternating); BENCH_ARGS: extra bench.py flags.
set -u
TAG=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
REPS=${REPS:-2}
for rep in $(seq 1 $REPS); do
  for lib in "$@"; do
    n=$(basename "$lib" .so)
    SG_LIB=$ROOT/$lib timeout -k 10 300 python bench.py --cpu-sample -1 --steps ${STEPS:-60} --warmup 10 ${BENCH_ARGS:-} \
      --json-out "$OUT/bench_${n}_$rep.json" > "$OUT/bench_${n}_$rep.log" 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "bench $n rc=$rc"; tail -5 "$OUT/bench_${n}_$rep.log"; exit $rc; }
    python -c "import json;d=json.load(open('$OUT/bench_${n}_$rep.json'));print('$n rep $rep', round(d['value']/1e6,1),'M pairs/s', round(d['ms_per_step'],4),'ms/step')"
  done
done
