#!/bin/bash
# Alternating A/B of run-time environment settings against the product defaults.
# Usage: scripts/gpu_env_ab.sh TAG "ENV=VAL [ENV2=VAL2]" ["..."]   (MODES as gpu_round5.sh)
set -u
TAG=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
run() {   # name, bench args, env settings...
  local name=$1 args=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --cpu-sample -1 $args --json-out "$OUT/$name.json" \
    > "$OUT/$name.log" 2>&1
  local rc=$?
  [ $rc -eq 0 ] || { echo "$name rc=$rc" | tee -a "$OUT/summary.txt"; exit $rc; }
  python -c "import json;d=json.load(open('$OUT/$name.json'));print('$name', round(d['value']/1e6,2),'M pairs/s', round(d['ms_per_step'],5),'ms/step')" | tee -a "$OUT/summary.txt"
}
for rep in 1 2; do
  for mode in ${MODES:-n1 emu8}; do
    case $mode in
      n1) A="--steps 40 --warmup 5" ;;
      emu8) A="--emulate-world 8 --steps 300 --warmup 30" ;;
      c3) A="--records bf16 --steps 40 --warmup 5" ;;
      avg) A="--stack average --steps 40 --warmup 5" ;;
      att) A="--stack attention --steps 40 --warmup 5" ;;
    esac
    run "prod_${mode}_$rep" "$A" SG_NOP=1
    k=0
    for e in "$@"; do k=$((k+1)); run "env${k}_${mode}_$rep" "$A" $e; done
  done
done
exit 0
