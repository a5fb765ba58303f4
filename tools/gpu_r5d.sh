#!/bin/bash
# Round-5 pass D: the GPU suite (with the full-size engine test), the config-4
# fused encode + HH256S sweep on this library (tools/sweep_fused.sh), and the
# RS(12,4) encode at an aligned shard length (S = 87040) beside the ragged
# 1 MiB block (S = 87382): what the rows' misalignment costs the GF sweep.
# Usage: bash tools/gpu_r5d.sh TAG
set -o pipefail
TAG=${1:-r5d}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -x -q --timeout 170 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 \
 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for sb in 1048576 1044480 1048576 1044480; do
  timeout -k 10 120 python -u bench.py --k 12 --m 4 --stripe-bytes $sb --steps 20 --no-extras --no-cpu-baseline > $OUT/enc12_$sb.json 2>/dev/null || exit 1
  tail -1 $OUT/enc12_$sb.json | cut -c1-120
done
bash tools/sweep_fused.sh $TAG/sweep > $OUT/sweep.log 2>&1 || { tail -5 $OUT/sweep.log; exit 1; }
echo done
