#!/bin/bash
# A/B of the vector GF kernels' workgroup size (RSG_VEC_BLOCK) through bench.py.
. "$(dirname "$0")/measure_env.sh"  # RSG_* knobs: the measurement build (ABI 6)
set -o pipefail
OUT=gpurun_out/ab_block
mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 20 --no-cpu-baseline > $OUT/b64_$i.json 2>>$OUT/err.log || exit $?
  RSG_VEC_BLOCK=256 timeout -k 10 120 python bench.py --steps 20 --no-cpu-baseline > $OUT/b256_$i.json 2>>$OUT/err.log || exit $?
done
timeout -k 10 120 python bench.py --steps 20 --no-cpu-baseline --no-extras --k 16 --m 4 > $OUT/b64_16_4.json 2>>$OUT/err.log || exit $?
RSG_VEC_BLOCK=256 timeout -k 10 120 python bench.py --steps 20 --no-cpu-baseline --no-extras --k 16 --m 4 > $OUT/b256_16_4.json 2>>$OUT/err.log || exit $?
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/ab_block/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    ex = d.get("extras", {})
    print(f.split("/")[-1], d["value"], d["roofline"]["kernel_ms_avg"], d["roofline"]["frac"],
          [ex[k]["ms"] for k in sorted(ex) if k.startswith("reconstruct")])
PY
