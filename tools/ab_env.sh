#!/bin/bash
# Interleaved A/B of environment knobs on one bench command.
# Usage: bash tools/ab_env.sh TAG "bench args" "ENV=a" "ENV=b" ...   (2 reps each)
set -o pipefail
TAG=$1; ARGS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  i=0
  for envs in "$@"; do
    i=$((i+1))
    env $envs timeout -k 10 120 python bench.py $ARGS > $OUT/v${i}_$rep.json 2>> $OUT/bench.err || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/v${i}_$rep.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$envs', 'rep $rep', r['kernel_ms_avg'], r['kernel_ms_min'], r['frac'])"
  done
done
