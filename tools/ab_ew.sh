#!/bin/bash
# A/B of the DMA fused encode+hash kernel's encoder shape: RSG_DMA_EW=4 (two
# encoder waves per stripe group, per-row folds) vs the default (one wave per
# group, generated XOR network).  Fused parity tests first, then interleaved
# bench --digests runs.  Usage: bash tools/ab_ew.sh TAG
. "$(dirname "$0")/measure_env.sh"  # RSG_* knobs: the measurement build (ABI 6)
set -o pipefail
TAG=${1:-ab_ew}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 170 --timeout-method thread -m gpu \
  tests/test_gpu_configs.py tests/test_gpu_parity.py -k "fused or config4 or dma" > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for rep in 1 2; do
  for ew in 4 2; do
    RSG_DMA_EW=$ew timeout -k 10 120 python bench.py --digests --steps 30 --warmup 3 --no-cpu-baseline --no-extras > $OUT/ew${ew}_$rep.json 2>> $OUT/bench.err || exit 1
    python3 -c "import json,sys; d=json.loads(open('$OUT/ew${ew}_$rep.json').read().strip().splitlines()[-1]); r=d['roofline']; print('EW=$ew rep $rep', r['kernel_ms_avg'], r['kernel_ms_min'], r['frac'])"
  done
done
