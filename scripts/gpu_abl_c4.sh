#!/bin/bash
# Timing ablations of the capacity-32 kernel (results invalid in the variants):
# C4 emulated W = 8 rank with the default library and each variant, alternating.
# Usage: scripts/gpu_abl_c4.sh TAG variant.so...
set -u
TAG=${1:-abl}; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  SG_LIB=$lib timeout -k 10 300 python bench.py --cpu-sample -1 "$@" --json-out "$OUT/$n.json" > "$OUT/$n.log" 2>&1
  local r=$?
  [ $r -eq 0 ] || { echo "$n rc=$r"; tail -5 "$OUT/$n.log"; exit $r; }
  python -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', round(d['value']/1e6,2),'M pairs/s', round(d['ms_per_step'],3),'ms')"
}
C4="--dataset syn_aids10knef --emulate-world 8 --steps 3 --warmup 1"
for rep in 1 2; do
  run c4_base_$rep graphembedding_amd/lib/libsiamese_hip.so $C4
  for v in "$@"; do run c4_$(basename $v .so)_$rep $v $C4; done
done
run c2_base graphembedding_amd/lib/libsiamese_hip.so --gpus 1 --steps 20 --warmup 5
run c2_base2 graphembedding_amd/lib/libsiamese_hip.so --gpus 1 --steps 20 --warmup 5
exit 0
