#!/bin/bash
# Round-4 pass Q: RS(10,4) (14-drive default) one-pass GET / heal with
# per-pattern XOR networks on four network waves (k_decode_records_net10):
# every listed pattern, the long ragged walks, then kernel stats against the
# run-time-table GET and the two-pass heal (RSG_DECODE_NET=0), interleaved.
# Usage: bash tools/gpu_r4q.sh TAG
set -o pipefail
TAG=${1:-r4q}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_decode_nets.py tests/test_gpu_decode.py tests/test_gpu_heal.py -x -q --timeout 170 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
cd /tmp
for round in 1 2; do
  for net in 1 0; do
    for what in into2 heal into1; do
      RSG_DECODE_NET=$net EP_K=10 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/n${net}_${round}_$what -o run --output-format csv -- python3 $R/tools/engine_prof.py $what 10 > $OUT/n${net}_${round}_$what.txt 2>&1 || exit $?
    done
  done
done
echo done
