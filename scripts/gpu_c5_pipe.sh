#!/bin/bash
# C5 chunk pipeline: GPU web tests, then the C5 bench with the pipeline on and off.
# Usage: scripts/gpu_c5_pipe.sh TAG
set -u
TAG=${1:-c5pipe}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_web.py > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --dataset syn_web --steps 3 --warmup 1 --cpu-sample -1 \
    --json-out "$OUT/$n.json" > "$OUT/$n.log" 2>&1
  local r=$?
  [ $r -eq 0 ] || { echo "$n rc=$r"; tail -5 "$OUT/$n.log"; exit $r; }
  python -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', round(d['value']/1e6,3),'M pairs/s', round(d['ms_per_step'],1),'ms')"
}
run pipe1 SG_WEB_PIPE=1
run pipe0 SG_WEB_PIPE=0
run pipe1b SG_WEB_PIPE=1
run pipe0b SG_WEB_PIPE=0
exit 0
