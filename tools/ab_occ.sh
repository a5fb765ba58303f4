#!/bin/bash
# A/B of the vector kernels' resident waves per SIMD (RSG_VEC_OCC).
. "$(dirname "$0")/measure_env.sh"  # RSG_* knobs: the measurement build (ABI 6)
set -o pipefail
OUT=gpurun_out/ab_occ2
mkdir -p $OUT
for occ in 0 2 3 1 0; do
  RSG_VEC_OCC=$occ timeout -k 10 120 python bench.py --steps 20 --no-cpu-baseline --no-engines > $OUT/occ$occ.json 2>>$OUT/err.log || exit $?
  RSG_VEC_OCC=$occ timeout -k 10 120 python bench.py --steps 20 --no-cpu-baseline --no-extras --k 16 --m 4 > $OUT/occ${occ}_16_4.json 2>>$OUT/err.log || exit $?
  python - $occ <<'PY'
import json, sys
o = sys.argv[1]
for suf in ("", "_16_4"):
    d = json.loads(open(f"gpurun_out/ab_occ2/occ{o}{suf}.json").read().strip().splitlines()[-1])
    ex = d.get("extras", {})
    print("occ", o, suf or "_8_4", d["roofline"]["kernel_ms_avg"], d["roofline"]["frac"],
          [ex[k]["kernel_ms"] for k in sorted(ex) if k.startswith("reconstruct")])
PY
done
