#!/bin/bash
# Round-3 GPU session: GPU tests, smoke, the driver's exact bench command, then a
# kernel-trace-only rocprof pass of that same command and separate PMC passes
# (HBM traffic; executed MFMA work).  Usage: scripts/gpu_round3.sh TAG [skip-tests]
# Outputs under gpurun_out/TAG; scripts/make_profile_summary.py condenses them.
set -u
TAG=${1:-run}
SKIP=${2:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
BENCH="bench.py --gpus 1 --steps 20 --warmup 5"
if [ -z "$SKIP" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest_gpu rc=$rc" | tee -a "$OUT/summary.txt"; tail -3 "$OUT/pytest_gpu.log"
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  rc=$?; echo "smoke rc=$rc" | tee -a "$OUT/summary.txt"
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python $BENCH --json-out "$OUT/bench.json" > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc" | tee -a "$OUT/summary.txt"; cat "$OUT/bench.json"
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
# kernel trace only (no PMC, no other tracing domains), same command minus the CPU leg
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --cpu-sample -1 \
  --json-out "$OUT/trace_bench.json" > "$OUT/trace.log" 2>&1
rc=$?; echo "rocprof trace rc=$rc" | tee -a "$OUT/summary.txt"
[ $rc -eq 0 ] || exit $rc
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
    "SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_MFMA_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE" \
    "SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp -d "$OUT/pmc$i" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --gpus 1 --steps 3 --warmup 1 --cpu-sample -1 > "$OUT/pmc$i.log" 2>&1
  rc=$?; echo "pmc$i [$grp] rc=$rc" | tee -a "$OUT/summary.txt"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
