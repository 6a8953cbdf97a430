#!/bin/bash
# Class-exclusive schedule: GPU tests of the order / parity paths, then the driver's bench
# command with the class schedule on and off (SG_CLASS_SCHEDULE), alternating, and a sweep
# of the class cost weights (SG_CLS_W).  Usage: scripts/gpu_cls_ab.sh TAG [weights...]
set -u
TAG=${1:-cls}; shift || true
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  ${TESTS:-tests/test_gpu_order.py tests/test_gpu_fullbatch.py tests/test_gpu_trajectory.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py} \
  > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
run() {   # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample -1 \
    --json-out "$OUT/bench_$n.json" > "$OUT/bench_$n.log" 2>&1
  local r=$?
  [ $r -eq 0 ] || { echo "bench $n rc=$r"; exit $r; }
  python -c "import json;d=json.load(open('$OUT/bench_$n.json'));print('$n', round(d['value']/1e6,1),'M pairs/s', round(d['ms_per_step'],4),'ms/step frac', round(d['roofline']['frac'],4))"
}
for rep in 1 2; do
  run cls_$rep SG_CLASS_SCHEDULE=1
  run mix_$rep SG_CLASS_SCHEDULE=0
done
i=0
for w in "$@"; do
  i=$((i+1))
  run w$i SG_CLASS_SCHEDULE=1 SG_CLS_W=$w
  echo "  weights $w"
done
exit 0
