#!/bin/bash
# Correctness, then encode rates for the rustfs geometries (per GPU, device-resident)
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/t.log 2>&1; tail -2 gpurun_out/t.log
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras"
for km in "8 4" "16 4" "12 4" "6 2" "6 6" "2 2" "4 2" "10 6" "8 8"; do
  set -- $km
  timeout -k 10 300 $B --k $1 --m $2 > gpurun_out/k_$1_$2.json 2>/dev/null || exit 1
  echo "RS($1,$2) $(python -c "import json; d=json.load(open('gpurun_out/k_$1_$2.json')); print(d['value'], d['roofline']['kernel_ms_avg'], d['roofline']['achieved'], d['roofline']['frac'])")"
done
