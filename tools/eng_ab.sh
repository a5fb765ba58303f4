#!/bin/bash
# GET / heal engine A/B: bench.py's engine extras per geometry and record
# engine (and optional label=env settings, e.g. SETS="gs1:RSG_GET_GS=1 gs2:RSG_GET_GS=2").
# Usage: [TAG=..] [GEOS="16,4 8,4"] [ENGINES="one-pass two-pass"] [SETS=...] bash tools/eng_ab.sh
set -o pipefail
OUT=gpurun_out/${TAG:-r3_eng_ab}; mkdir -p $OUT
for geo in ${GEOS:-16,4 8,4}; do
 k=${geo%,*}; m=${geo#*,}
 for e in ${ENGINES:-one-pass two-pass}; do
 for set in ${SETS:-default:}; do
  lab=${set%%:*}; envs=${set#*:}; envs=${envs//,/ }
  env $envs timeout -k 10 200 python -u bench.py --k $k --m $m --no-cpu-baseline --no-config-extras --record-engine $e --steps 5 > $OUT/k${k}_${e}_$lab.json 2> $OUT/k${k}_${e}_$lab.err || exit $?
  python - $OUT/k${k}_${e}_$lab.json $k $e $lab <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); g=d['extras']['engines']
print(sys.argv[2], sys.argv[3], sys.argv[4], {k:(v.get('kernel_ms'),v['frac']) for k,v in g.items() if isinstance(v,dict)}, flush=True)
PY
 done
 done
done
