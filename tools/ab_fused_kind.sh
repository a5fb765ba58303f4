#!/bin/bash
# Config 4 at SURVEY's 4 GiB sizing: every fused-kernel kind (auto = the
# launcher's choice, ring, wide2, wide4, dma) for the few-large-stripe points
# (2, 4, 8, 16 MiB stripes, n = 4 GiB / stripe), one process per kind (the
# kind is read once per process).  Output: gpurun_out/<TAG>/<kind>_<MiB>m.json
# Usage: [SIZES="1 2 4 8 16"] bash tools/ab_fused_kind.sh TAG [kinds...]  (1 MiB: n = 4096)
. "$(dirname "$0")/measure_env.sh"  # RSG_* knobs: the measurement build (ABI 6)
set -o pipefail
TAG=${1:-ab_kind}; shift
KINDS=${@:-auto ring wide2 wide4 dma}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for mib in ${SIZES:-2 4 8 16}; do
  bytes=$((mib * 1024 * 1024))
  n=$((4096 / mib)); [ "$n" -lt 4096 ] || n=4096
  for kind in $KINDS; do
    if [ "$kind" = auto ]; then env=""; else env="RSG_FUSED_KIND=$kind"; fi
    env $env timeout -k 10 120 python bench.py --stripe-bytes $bytes --batch $n --digests --steps 10 --warmup 3 \
        --no-extras --no-cpu-baseline --no-config-extras > $OUT/${kind}_${mib}m.json 2> $OUT/${kind}_${mib}m.err || exit $?
    python - $OUT/${kind}_${mib}m.json $kind $mib <<'EOF'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"]
print(f"{sys.argv[3]:>2} MiB n={d['config']['stripes_per_gpu']:5d} {sys.argv[2]:6s} kernel {r['kernel_ms_avg']:.3f} ms (min {r['kernel_ms_min']:.3f}) frac {r['frac']:.3f}", flush=True)
EOF
  done
done
