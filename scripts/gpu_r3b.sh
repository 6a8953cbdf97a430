#!/bin/bash
# Round-3 A/B session: C5 parity tests, C5 bench with the XCD-partitioned unit order on
# and off (SG_WEB_XCD), a per-wave timing pass of the headline kernel, and headline
# bench lines for library variants / class weights.  Usage:
#   scripts/gpu_r3b.sh TAG [lib.so ...]      (CLS_WEIGHTS="w0,w1,w2,w3 ..." optional)
set -u
TAG=${1:-r3b}; shift || true
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  ${TESTS:-tests/test_gpu_web.py} > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
c5() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --dataset syn_web --steps 3 --warmup 1 --cpu-sample -1 \
    --json-out "$OUT/c5_$n.json" > "$OUT/c5_$n.log" 2>&1
  local r=$?
  [ $r -eq 0 ] || { echo "c5 $n rc=$r"; tail -5 "$OUT/c5_$n.log"; exit $r; }
  python -c "import json;d=json.load(open('$OUT/c5_$n.json'));print('c5 $n', round(d['value']/1e6,3),'M pairs/s', round(d['ms_per_step'],1),'ms')"
}
if [ -z "${SKIP_C5:-}" ]; then
  for rep in 1 2; do
    c5 xcd_$rep SG_WEB_XCD=1
    c5 flat_$rep SG_WEB_XCD=0
  done
fi
if [ -f graphembedding_amd/lib/libsiamese_timing.so ] && [ -z "${SKIP_TIMING:-}" ]; then
  SG_LIB=$ROOT/graphembedding_amd/lib/libsiamese_timing.so timeout -k 10 300 \
    python scripts/fast_timing.py 1 8 > "$OUT/timing.log" 2>&1
  rc=$?; echo "timing rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
hb() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample -1 \
    --json-out "$OUT/c2_$n.json" > "$OUT/c2_$n.log" 2>&1
  local r=$?
  [ $r -eq 0 ] || { echo "c2 $n rc=$r"; tail -5 "$OUT/c2_$n.log"; exit $r; }
  python -c "import json;d=json.load(open('$OUT/c2_$n.json'));print('c2 $n', round(d['value']/1e6,1),'M pairs/s', round(d['ms_per_step'],4),'ms frac', round(d['roofline']['frac'],4))"
}
for rep in 1 2; do
  hb base_$rep
  for lib in "$@"; do
    hb "$(basename "$lib" .so)_$rep" SG_LIB=$ROOT/$lib
  done
  i=0
  for w in ${CLS_WEIGHTS:-}; do
    i=$((i+1)); hb w${i}_$rep SG_CLS_W=$w
  done
done
echo "weights: ${CLS_WEIGHTS:-}"
exit 0
