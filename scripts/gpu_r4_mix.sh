#!/bin/bash
# Round 4 combined GPU run: C4 tests + C4 A/B (new tree vs var_c4_orig.so), then the C5
# script (TKG A/B + pipeline-off trace + PMC).  Usage: scripts/gpu_r4_mix.sh TAG
set -u
TAG=${1:-r04_mix}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd "$ROOT"
TESTS="tests/test_gpu_fast32.py tests/test_gpu_trainshape.py::test_c4_store_sourced_training_launch tests/test_gpu_source.py" \
BENCH_ARGS="--dataset syn_aids10knef --steps 3 --warmup 1" REPS=2 \
  bash scripts/gpu_var.sh ${TAG}_c4 new= old=SG_LIB=graphembedding_amd/lib/var_c4_orig.so || exit $?
bash scripts/gpu_r4_c5.sh ${TAG}_c5 SG_WEB_TKG=0 || exit $?
