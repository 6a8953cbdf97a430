#!/bin/bash
# C5 A/B: the C5 GPU tests, then the C5 bench for each variant, alternating over REPS
# rounds.  A variant is NAME=ENV1,ENV2,... (environment assignments, e.g.
# SG_LIB=graphembedding_amd/lib/x.so or SG_WEB_XCD=0; "base=" for none).
# Usage: scripts/gpu_c5_var.sh TAG variant...
set -u
TAG=${1:-c5var}; shift || true
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    ${TESTS:-tests/test_gpu_web.py tests/test_gpu_fullsize.py::test_c5_web_sampled_pairs} \
    > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"
  [ $rc -eq 0 ] || exit $rc
fi
for rep in $(seq 1 ${REPS:-2}); do
  for v in "$@"; do
    n=${v%%=*}; e=${v#*=}
    envs=$(echo "$e" | tr ',' ' ')
    env $envs timeout -k 10 300 python bench.py --dataset syn_web --steps 3 --warmup 1 --cpu-sample -1 \
      ${BENCH_ARGS:-} --json-out "$OUT/${n}_$rep.json" > "$OUT/${n}_$rep.log" 2>&1
    r=$?
    [ $r -eq 0 ] || { echo "$n rc=$r"; tail -5 "$OUT/${n}_$rep.log"; exit $r; }
    python -c "import json;d=json.load(open('$OUT/${n}_$rep.json'));print('$n rep $rep', round(d['value']/1e6,3),'M pairs/s', round(d['ms_per_step'],1),'ms')"
  done
done
exit 0
