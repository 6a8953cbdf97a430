#!/bin/bash
# Round 4: fused Attention pooling — parity tests, then bench lines of the three stacks.
set -u
OUT=gpurun_out/${1:-r04_att}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_order.py \
  tests/test_gpu_source.py tests/test_gpu_fullbatch.py -x -v -m gpu --timeout 300 \
  --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
for st in attention average default; do
  timeout -k 10 300 python bench.py --stack $st --steps 20 --warmup 5 --cpu-sample -1 \
    --json-out "$OUT/bench_$st.json" > "$OUT/bench_$st.log" 2>&1
  rc=$?; echo "bench $st rc=$rc"; cat "$OUT/bench_$st.json"
  [ $rc -eq 0 ] || exit $rc
done
