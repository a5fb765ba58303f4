#!/bin/bash
# A/B of the network GET/heal kernel's knobs: bench.py's engine extras per
# environment setting.  Usage: bash tools/ab_net.sh TAG "ENV1" "ENV2" ...
set -o pipefail
TAG=${1:-r3_ab_net}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
i=0
for envs in "$@"; do
  i=$((i+1))
  env $envs timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-config-extras --steps 5 $BENCH_ARGS > $OUT/ab$i.json 2> $OUT/ab$i.err || exit $?
  python - $OUT/ab$i.json "$envs" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); g=d['extras']['engines']
print(sys.argv[2], {k:(v.get('kernel_ms'),v['frac']) for k,v in g.items() if isinstance(v,dict) and 'bitrot' not in k}, flush=True)
PY
done
