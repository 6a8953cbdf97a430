#!/bin/bash
# Round-4 end-of-round GPU session: scripts/gpu_round3.sh (GPU tests, smoke, the driver's
# bench command, its kernel-trace-only rocprof pass and the PMC passes), then the config
# sweep.  Usage: scripts/gpu_round4.sh TAG [skip-tests]
set -u
TAG=${1:-r04_final}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
bash "$ROOT/scripts/gpu_round3.sh" "$TAG" ${2:-} || exit $?
bash "$ROOT/scripts/config_sweep.sh" "${TAG}_sweep" || exit $?
exit 0
