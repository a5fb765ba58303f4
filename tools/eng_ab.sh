#!/bin/bash
set -o pipefail
OUT=gpurun_out/r3_eng_ab; mkdir -p $OUT
for geo in "16 4" "8 4"; do set -- $geo
 for e in one-pass two-pass; do
  timeout -k 10 200 python -u bench.py --k $1 --m $2 --no-cpu-baseline --no-config-extras --record-engine $e --steps 5 > $OUT/k$1_$e.json 2> $OUT/k$1_$e.err || exit $?
  python - $OUT/k$1_$e.json $1 $e <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); g=d['extras']['engines']
print(sys.argv[2], sys.argv[3], {k:(v.get('kernel_ms'),v['frac']) for k,v in g.items() if isinstance(v,dict)})
PY
 done
done
