#!/bin/bash
# A/B of the hash kernel's prefetch depth (RSG_HASH_DEPTH = batches of 8
# packets in flight per lane) on the record engines (bench.py extras:
# GET, heal, bitrot_verify) and the fused-digest fallback paths.
. "$(dirname "$0")/measure_env.sh"  # RSG_* knobs: the measurement build (ABI 6)
set -o pipefail
OUT=gpurun_out/ab_hash
mkdir -p $OUT
for d in 2 3 1 2 3; do
  RSG_HASH_DEPTH=$d timeout -k 10 120 python bench.py --steps 5 --no-cpu-baseline > $OUT/d$d.json 2>>$OUT/err.log || exit $?
  python - $d <<'PY'
import json, sys
d = sys.argv[1]
x = json.loads(open(f"gpurun_out/ab_hash/d{d}.json").read().strip().splitlines()[-1])["extras"]["engines"]
print("depth", d, {k: v["call_ms"] for k, v in x.items()})
PY
done
