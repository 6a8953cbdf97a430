#!/bin/bash
set -u
OUT=gpurun_out/r06_ff; mkdir -p $OUT
for rep in 1 2; do
  for sm in 60 250 1000; do
    timeout -k 10 300 python bench.py --cpu-sample -1 --settle-ms $sm --json-out $OUT/s${sm}_$rep.json > $OUT/s${sm}_$rep.log 2>&1 || exit 1
    python -c "import json;d=json.load(open('$OUT/s${sm}_$rep.json'));print('settle $sm rep $rep', round(d['value']/1e6,2), round(d['ms_per_step'],5))" | tee -a $OUT/summary.txt
  done
done
