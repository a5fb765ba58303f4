#!/bin/bash
# Round-4 pass S: verify-hash batch depth (RSG_HASH_DEPTH = 2 default, 3) on
# the all-present GET of the geometries whose records are not 8-aligned
# (RS(10,4), RS(12,4): 2 mod 8; RS(6,4): odd) and RS(8,4), interleaved.
# Usage: bash tools/gpu_r4s.sh TAG
set -o pipefail
TAG=${1:-r4s}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for round in 1 2; do
  for d in 2 3; do
    for k in 10 12 6 8; do
      RSG_HASH_DEPTH=$d EP_K=$k timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/d${d}_${round}_k$k -o run --output-format csv -- python3 $R/tools/engine_prof.py into0 10 > $OUT/d${d}_${round}_k$k.txt 2>&1 || exit $?
    done
  done
done
echo done
