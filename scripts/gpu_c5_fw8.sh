#!/bin/bash
# C5 forward instance kernel at 8 waves (room for the pipelined GEMMs): bench A/B.
set -u
TAG=${1:-c5fw8}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --dataset syn_web --steps 3 --warmup 1 --cpu-sample -1 \
    --json-out "$OUT/$n.json" > "$OUT/$n.log" 2>&1
  local r=$?
  [ $r -eq 0 ] || { echo "$n rc=$r"; tail -5 "$OUT/$n.log"; exit $r; }
  python -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', round(d['value']/1e6,3),'M pairs/s', round(d['ms_per_step'],1),'ms')"
}
L8=graphembedding_amd/lib/libsiamese_fw8.so
run base SG_WEB_PIPE=1
run fw8_pipe_bpc1 SG_LIB=$L8 SG_WEB_PIPE=1 SG_WEB_FWD_BPC=1
run fw8_pipe SG_LIB=$L8 SG_WEB_PIPE=1
run fw8_nopipe SG_LIB=$L8 SG_WEB_PIPE=0
run base_nopipe_bpc1 SG_WEB_PIPE=0 SG_WEB_FWD_BPC=1
run fw8_nopipe_bpc1 SG_LIB=$L8 SG_WEB_PIPE=0 SG_WEB_FWD_BPC=1
exit 0
