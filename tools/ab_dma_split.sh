#!/bin/bash
# Fused DMA kernel (RS(8,4), n >= 2048): one encoder wave per 4-stripe group
# (default) vs two taking alternate steps (RSG_DMA_EW=4), 1 and 2 MiB stripes.
. "$(dirname "$0")/measure_env.sh"  # RSG_* knobs: the measurement build (ABI 6)
set -o pipefail
OUT=gpurun_out/${TAG:-ab_dma_split}; mkdir -p $OUT
for rep in 1 2; do
for cfg in "1048576 4096" "2097152 2048"; do set -- $cfg
  for ew in 2 4; do
    RSG_DMA_EW=$ew timeout -k 10 120 python bench.py --stripe-bytes $1 --batch $2 --digests --steps 20 --warmup 3 \
      --no-extras --no-cpu-baseline --no-config-extras > $OUT/ew${ew}_$2_r$rep.json 2> $OUT/ew${ew}_$2_r$rep.err || exit $?
    python -c "import json,sys; d=json.loads([l for l in open('$OUT/ew${ew}_$2_r$rep.json') if l.startswith('{')][-1]); r=d['roofline']; print('n=$2 ew=$ew rep=$rep', r['kernel_ms_avg'], r['kernel_ms_min'], r['frac'], flush=True)"
  done
done
done
