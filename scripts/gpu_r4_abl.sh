#!/bin/bash
# Round 4: C5 forward timing ablations (results invalid; libraries built with
# SG_TIMING_ABLATION_BUILD), each under a kernel trace with the pipeline off, then the C4
# PMC passes.  Usage: scripts/gpu_r4_abl.sh TAG
set -u
TAG=${1:-r04_abl}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in base FHASH FH1 FH2; do
  if [ $v = base ]; then LIBENV=""; else LIBENV="$ROOT/graphembedding_amd/lib/abl_$v.so"; fi
  SG_LIB=$LIBENV SG_WEB_PIPE=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/$v" -o run \
    --output-format csv -- python3 "$ROOT/bench.py" --dataset syn_web --steps 1 --warmup 1 \
    --cpu-sample -1 --json-out "$OUT/$v.json" > "$OUT/$v.log" 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 - "$OUT/$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'web_gcn' in r['Name']:
        print('   ', r['Name'].split('(')[0].replace('void (anonymous namespace)::', ''),
              'avg', round(float(r['AverageNs']) / 1e6, 3), 'max', round(float(r['MaxNs']) / 1e6, 3))
PY
done
cd "$ROOT"
bash scripts/gpu_pmc_c4.sh ${TAG}_pmc4 > "$OUT/pmc4.txt" 2>&1
rc=$?; echo "pmc4 rc=$rc"; tail -30 "$OUT/pmc4.txt"
