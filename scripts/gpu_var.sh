#!/bin/bash
# Bench A/B over variants, alternating over REPS rounds.  A variant is NAME=ENV1+ENV2+...
# (environment assignments joined by '+', such as SG_LIB=graphembedding_amd/lib/x.so; "base=" for none).
# BENCH_ARGS: the bench.py flags (default: the driver's command, --gpus 1 --steps 20
# --warmup 5).  TESTS (optional): pytest targets run first, with TEST_ENV applied.
# Usage: scripts/gpu_var.sh TAG variant...
set -u
TAG=${1:-var}; shift || true
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
if [ -n "${TESTS:-}" ]; then
  env ${TEST_ENV:-} timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    -m gpu $TESTS > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"
  [ $rc -eq 0 ] || exit $rc
fi
ARGS=${BENCH_ARGS:---gpus 1 --steps 20 --warmup 5}
for rep in $(seq 1 ${REPS:-2}); do
  for v in "$@"; do
    n=${v%%=*}; e=${v#*=}
    envs=$(echo "$e" | tr '+' ' ')
    env $envs timeout -k 10 300 python bench.py $ARGS --cpu-sample -1 \
      --json-out "$OUT/${n}_$rep.json" > "$OUT/${n}_$rep.log" 2>&1
    r=$?
    [ $r -eq 0 ] || { echo "$n rc=$r"; tail -5 "$OUT/${n}_$rep.log"; exit $r; }
    python -c "import json;d=json.load(open('$OUT/${n}_$rep.json'));print('$n rep $rep', round(d['value']/1e6,3),'M pairs/s', round(d['ms_per_step'],4),'ms frac', round(d['roofline']['frac'],4))"
  done
done
exit 0
