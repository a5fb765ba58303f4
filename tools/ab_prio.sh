#!/bin/bash
# A/B of wave priorities: one-pass GET/heal kernels (RSG_DMA_PRIO) and the
# DMA fused encode+hash kernel (RSG_ENC_PRIO).
. "$(dirname "$0")/measure_env.sh"  # RSG_* knobs: the measurement build (ABI 6)
set -o pipefail
OUT=gpurun_out/ab_prio2
mkdir -p $OUT
for v in 2 0 2 0; do
  RSG_DMA_PRIO=$v timeout -k 10 120 python bench.py --steps 5 --no-cpu-baseline > $OUT/p$v.json 2>>$OUT/err.log || exit $?
  python - $v <<'PY'
import json, sys
v = sys.argv[1]
x = json.loads(open(f"gpurun_out/ab_prio2/p{v}.json").read().strip().splitlines()[-1])["extras"]["engines"]
print("dma prio", v, {k: x[k]["call_ms"] for k in ("get_2_data_lost", "heal_1data_1parity")})
PY
done
for v in 0 1 2 3 0 2; do
  RSG_ENC_PRIO=$v timeout -k 10 120 python bench.py --digests --steps 10 --no-cpu-baseline --no-extras > $OUT/e$v.json 2>>$OUT/err.log || exit $?
  python - $v <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open(f"gpurun_out/ab_prio2/e{v}.json").read().strip().splitlines()[-1])
print("enc prio", v, d["roofline"]["kernel_ms_avg"], d["roofline"]["frac"])
PY
done
