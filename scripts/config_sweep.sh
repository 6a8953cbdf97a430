#!/bin/bash
# One bench line per BASELINE config on 1 GPU (+ emulated per-rank W=8 lines).
# Usage: scripts/config_sweep.sh TAG
set -u
TAG=${1:-sweep}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" --json-out "$OUT/$name.json" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
run c2_n1 --cpu-sample -1
run c2_emu8 --emulate-world 8 --steps 200 --warmup 20 --cpu-sample -1
run c2_emu8c --emulate-world 8 --emulate-collective --steps 200 --warmup 20 --cpu-sample -1
run c3_n1 --records bf16 --cpu-sample -1
run c3_emu8 --records bf16 --emulate-world 8 --steps 200 --warmup 20 --cpu-sample -1
run c4_n1 --dataset syn_aids10knef --steps 3 --warmup 1 --cpu-sample -1
run c4_emu8 --dataset syn_aids10knef --emulate-world 8 --steps 3 --warmup 1 --cpu-sample -1
run c5_n1 --dataset syn_web --steps 3 --warmup 1 --cpu-sample -1
run c5_emu8 --dataset syn_web --emulate-world 8 --steps 3 --warmup 1 --cpu-sample -1
run avg_n1 --stack average --cpu-sample -1
run avg_emu8 --stack average --emulate-world 8 --steps 200 --warmup 20 --cpu-sample -1
run att_n1 --stack attention --cpu-sample -1
run att_emu8 --stack attention --emulate-world 8 --steps 200 --warmup 20 --cpu-sample -1
exit 0
