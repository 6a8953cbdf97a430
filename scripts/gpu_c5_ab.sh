#!/bin/bash
# C5 (Web-sized graphs): GPU tests of the graph-store path, then the C5 bench with the
# instance units on and off (SG_WEB_UNITS), alternating.  Usage: scripts/gpu_c5_ab.sh TAG
set -u
TAG=${1:-c5}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  ${TESTS:-tests/test_gpu_web.py tests/test_gpu_fullsize.py::test_c5_web_sampled_pairs} \
  > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
run() {   # name env...
  local n=$1; shift
  env "$@" timeout -k 10 400 python bench.py --dataset syn_web --steps 3 --warmup 1 --cpu-sample -1 \
    --json-out "$OUT/bench_$n.json" > "$OUT/bench_$n.log" 2>&1
  local r=$?
  [ $r -eq 0 ] || { echo "bench $n rc=$r"; tail -5 "$OUT/bench_$n.log"; exit $r; }
  python -c "import json;d=json.load(open('$OUT/bench_$n.json'));print('$n', round(d['value']/1e6,3),'M pairs/s', round(d['ms_per_step'],1),'ms/step frac', round(d['roofline']['frac'],4))"
}
for rep in 1 2; do
  run units_$rep SG_WEB_UNITS=1
  run single_$rep SG_WEB_UNITS=0
done
exit 0
