#!/bin/bash
# GET engine GF-pass time vs occupancy cap (RSG_VEC_OCC) through the C ABI.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/gep3
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for OCC in 0 1 2; do
  RSG_VEC_OCC=$OCC timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT -o occ$OCC -- $GRAFT_REPO_ROOT/tools/kbench/get_engine_probe 4096 3 4 > $OUT/occ$OCC.txt 2>&1 || exit $?
done
