#!/bin/bash
# GET / heal engine A/B: bench.py's engine extras per geometry and record
# engine.  Usage: [TAG=..] [GEOS="16,4 8,4"] [ENGINES="one-pass two-pass"] bash tools/eng_ab.sh
set -o pipefail
OUT=gpurun_out/${TAG:-r3_eng_ab}; mkdir -p $OUT
for geo in ${GEOS:-16,4 8,4}; do
 k=${geo%,*}; m=${geo#*,}
 for e in ${ENGINES:-one-pass two-pass}; do
  timeout -k 10 200 python -u bench.py --k $k --m $m --no-cpu-baseline --no-config-extras --record-engine $e --steps 5 > $OUT/k${k}_$e.json 2> $OUT/k${k}_$e.err || exit $?
  python - $OUT/k${k}_$e.json $k $e <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); g=d['extras']['engines']
print(sys.argv[2], sys.argv[3], {k:(v.get('kernel_ms'),v['frac']) for k,v in g.items() if isinstance(v,dict)}, flush=True)
PY
 done
done
