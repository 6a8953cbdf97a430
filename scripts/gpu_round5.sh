#!/bin/bash
# Round-5 GPU session: the GPU suite + smoke on the product library, an alternating A/B of
# C2 at N = 1 and at an emulated W = 8 rank (product library, variant libraries under ab/,
# and class-weight settings through SG_CLS_W), then the driver's bench command with its
# kernel-trace and PMC passes (scripts/gpu_round3.sh).  Usage:
#   scripts/gpu_round5.sh TAG [skip-tests]    (variants: VARIANTS="ab/x.so ab/y.so",
#                                              CLSW="1,1.315,1.316,1.493 ...",
#                                              XCDW="10000,10000,... (8) ...",
#                                              MODES="n1 emu8 n1ea emu8ea c4 c5 c3 avg att")
set -u
TAG=${1:-r05}
SKIP=${2:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
if [ -z "$SKIP" ]; then
  timeout -k 10 600 python -u -m pytest tests -v -m gpu --timeout 240 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest_gpu rc=$rc" | tee -a "$OUT/summary.txt"; tail -3 "$OUT/pytest_gpu.log"
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  rc=$?; echo "smoke rc=$rc" | tee -a "$OUT/summary.txt"
  [ $rc -eq 0 ] || exit $rc
fi
ab() {   # name, env-prefix..., -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --cpu-sample -1 ${BENCH_ARGS_AB:-} \
    --json-out "$OUT/ab_$name.json" > "$OUT/ab_$name.log" 2>&1
  local rc=$?
  [ $rc -eq 0 ] || { echo "ab $name rc=$rc" | tee -a "$OUT/summary.txt"; exit $rc; }
  python -c "import json;d=json.load(open('$OUT/ab_$name.json'));print('$name', round(d['value']/1e6,2),'M pairs/s', round(d['ms_per_step'],5),'ms/step')" | tee -a "$OUT/summary.txt"
}
for rep in 1 2; do
  for mode in ${MODES:-n1 emu8}; do
    case $mode in
      n1) BENCH_ARGS_AB="--steps 40 --warmup 5" ;;
      emu8) BENCH_ARGS_AB="--emulate-world 8 --steps 300 --warmup 30" ;;
      n1sep) BENCH_ARGS_AB="--steps 40 --warmup 5 --no-fused-adam" ;;
      emu8sep) BENCH_ARGS_AB="--emulate-world 8 --steps 300 --warmup 30 --no-fused-adam" ;;
      emu8c) BENCH_ARGS_AB="--emulate-world 8 --emulate-collective --steps 300 --warmup 30" ;;
      n1ea) BENCH_ARGS_AB="--steps 40 --warmup 5 --events after" ;;
      emu8ea) BENCH_ARGS_AB="--emulate-world 8 --steps 300 --warmup 30 --events after" ;;
      c4) BENCH_ARGS_AB="--dataset syn_aids10knef --steps 2 --warmup 1" ;;
      c5) BENCH_ARGS_AB="--dataset syn_web --steps 3 --warmup 1" ;;
      c3) BENCH_ARGS_AB="--records bf16 --steps 40 --warmup 5" ;;
      avg) BENCH_ARGS_AB="--stack average --steps 40 --warmup 5" ;;
      att) BENCH_ARGS_AB="--stack attention --steps 40 --warmup 5" ;;
    esac
    ab "prod_${mode}_$rep" SG_NOP=1
    for v in ${VARIANTS:-}; do ab "$(basename $v .so)_${mode}_$rep" SG_LIB=$ROOT/$v; done
    k=0
    for w in ${CLSW:-}; do k=$((k+1)); ab "clsw${k}_${mode}_$rep" SG_CLS_W=$w; done
    k=0
    for w in ${XCDW:-}; do k=$((k+1)); ab "xcdw${k}_${mode}_$rep" SG_XCD_W=$w; done
  done
done
[ -n "${NO_ROUND3:-}" ] && exit 0
bash scripts/gpu_round3.sh "$TAG" skip > "$OUT/round3.log" 2>&1
rc=$?; echo "gpu_round3 rc=$rc" | tee -a "$OUT/summary.txt"
exit $rc
