#!/bin/bash
# Interleaved A/B of environment knobs on the GET / heal engine extras of
# bench.py (kernel_ms per engine call).  Usage: bash tools/ab_eng.sh TAG "ENV=a" "ENV=b" ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  i=0
  for envs in "$@"; do
    i=$((i+1))
    env $envs timeout -k 10 180 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/v${i}_$rep.json 2>> $OUT/bench.err || exit 1
    python3 -c "
import json; d=json.loads(open('$OUT/v${i}_$rep.json').read().strip().splitlines()[-1]); e=d['extras']['engines']
print('$envs', 'rep $rep', ' '.join(f\"{k}={v.get('kernel_ms')}/{v['frac']}\" for k,v in e.items()))"
  done
done
