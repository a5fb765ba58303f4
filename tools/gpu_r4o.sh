#!/bin/bash
# Round-4 pass O: the verify hash on unaligned messages with aligned loads and
# a funnel shift (k_hh256_quad<0, 2, UNAL>) against unaligned 8-byte loads
# (RSG_HASH_UNAL=0): the GPU suite's record / hash tests, then the
# all-present GET (k data records verified) of RS(6,4), RS(10,4), RS(12,4) and
# RS(8,4) interleaved A B A B.  Usage: bash tools/gpu_r4o.sh TAG
set -o pipefail
TAG=${1:-r4o}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -x -q --timeout 170 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
cd /tmp
for round in 1 2; do
  for u in 1 0; do
    for k in 6 10 12 8; do
      RSG_HASH_UNAL=$u EP_K=$k timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/u${u}_${round}_k$k -o run --output-format csv -- python3 $R/tools/engine_prof.py into0 10 > $OUT/u${u}_${round}_k$k.txt 2>&1 || exit $?
    done
  done
done
echo done
