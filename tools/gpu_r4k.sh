#!/bin/bash
# Round-4 pass K: RS(12,4) GET with a 2-slot ring and two workgroups per CU
# (RSG_NET12_RD=2) against the 4-slot ring with one (default): the RS(12,4)
# pattern tests under the 2-slot build, then kernel stats interleaved A B A B.
# Usage: bash tools/gpu_r4k.sh TAG
set -o pipefail
TAG=${1:-r4k}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
RSG_NET12_RD=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_decode_nets.py -x -q --timeout 170 --timeout-method thread -m gpu -k "rs12 or ragged" > $OUT/pytest_rd2.log 2>&1 || { tail -40 $OUT/pytest_rd2.log; exit 1; }
tail -2 $OUT/pytest_rd2.log
cd /tmp
for round in 1 2; do
  for rd in 4 2; do
    for what in into2 into1; do
      RSG_NET12_RD=$rd EP_K=12 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/rd${rd}_${round}_$what -o run --output-format csv -- python3 $R/tools/engine_prof.py $what 10 > $OUT/rd${rd}_${round}_$what.txt 2>&1 || exit $?
    done
  done
done
echo done
