#!/bin/bash
# Encode bench over geometries (1 MiB stripes, n=4096), one GPU; each step
# under its own time limit.  Output: gpurun_out/$TAG/geom_k_${k}_${m}.json
set -o pipefail
TAG=${1:-geom}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for km in "16 4" "12 4" "10 6" "8 8" "6 6" "8 4" "4 2" "2 2" "6 2"; do
  set -- $km
  timeout -k 10 300 python bench.py --k $1 --m $2 --steps 20 --warmup 3 --no-cpu-baseline --no-extras > $OUT/geom_k_$1_$2.json 2>>$OUT/err.log || exit $?
done
