#!/bin/bash
# Headline A/B: the default bench line without extras, per environment
# setting (encode kernel_ms and frac; RS(16,4) with BENCH_ARGS).
# Usage: [BENCH_ARGS=...] bash tools/ab_headline.sh TAG "ENV1" "ENV2" ...
set -o pipefail
TAG=${1:-r3_ab_head}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
i=0
for envs in "$@"; do
  i=$((i+1))
  env $envs timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-extras --steps 30 $BENCH_ARGS > $OUT/h$i.json 2> $OUT/h$i.err || exit $?
  python - $OUT/h$i.json "$envs" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']
print(sys.argv[2], r['kernel_ms_avg'], r['kernel_ms_min'], r['frac'], flush=True)
PY
done
