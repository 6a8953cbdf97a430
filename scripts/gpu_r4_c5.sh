#!/bin/bash
# Round 4, C5: graph-store GPU tests, the C5 bench A/B of one switch (VAR_ENV, e.g.
# SG_WEB_TKG=0) against the default, then the pipeline-off kernel trace and two PMC passes
# (issue / wait counters; FETCH_SIZE) of one C5 step, summarised by scripts/pmc_c5_summary.py.
# Usage: scripts/gpu_r4_c5.sh TAG [VAR_ENV]
set -u
TAG=${1:-r04_c5}
VAR=${2:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    ${TESTS:-tests/test_gpu_web.py} > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
fi
run() {   # name env...
  local n=$1; shift
  env "$@" timeout -k 10 400 python bench.py --dataset syn_web --steps 3 --warmup 1 --cpu-sample -1 \
    --json-out "$OUT/bench_$n.json" > "$OUT/bench_$n.log" 2>&1
  local r=$?
  [ $r -eq 0 ] || { echo "bench $n rc=$r"; tail -5 "$OUT/bench_$n.log"; exit $r; }
  python -c "import json;d=json.load(open('$OUT/bench_$n.json'));print('$n', round(d['value']/1e6,3),'M pairs/s', round(d['ms_per_step'],1),'ms/step frac', round(d['roofline']['frac'],4))"
}
for rep in 1 2; do
  run new_$rep SG_WEB_X=1
  [ -n "$VAR" ] && run var_$rep $VAR
done
[ "${SKIP_PROF:-0}" = 1 ] && exit 0
cd /tmp && export TMPDIR=/tmp
export SG_WEB_PIPE=0
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --dataset syn_web --steps 1 --warmup 1 --cpu-sample -1 > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 400 rocprofv3 --pmc $grp -d "$OUT/pmc$i" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --dataset syn_web --steps 1 --warmup 1 --cpu-sample -1 > "$OUT/pmc$i.log" 2>&1
  rc=$?; echo "pmc$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 "$ROOT/scripts/pmc_c5_summary.py" "$OUT" > "$OUT/pmc_summary.txt" 2>&1
cat "$OUT/pmc_summary.txt"
exit 0
