#!/bin/bash
# Round-4 pass L: RS(8,4) GET / heal with four network waves, 4-stripe
# workgroups and two workgroups per CU (k_decode_records_net8q, default)
# against the two-wave 8-stripe kernel (RSG_NET8Q=0): every RS(8,4) pattern
# and the long / ragged walks, then kernel stats interleaved A B A B.
# Usage: bash tools/gpu_r4l.sh TAG
set -o pipefail
TAG=${1:-r4l}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_decode_nets.py tests/test_gpu_decode.py tests/test_gpu_heal.py tests/test_gpu_async.py -x -q --timeout 170 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
cd /tmp
for round in 1 2; do
  for q in 1 0; do
    for what in into2 heal into1; do
      RSG_NET8Q=$q EP_K=8 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/q${q}_${round}_$what -o run --output-format csv -- python3 $R/tools/engine_prof.py $what 10 > $OUT/q${q}_${round}_$what.txt 2>&1 || exit $?
    done
  done
done
echo done
