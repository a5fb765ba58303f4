#!/bin/bash
# Round-4 pass R: RS(4,4) (8-drive default) one-pass GET / heal with
# per-pattern XOR networks (k_decode_records_net4): the whole GPU suite and
# smoke on the library as shipped, then kernel stats against the
# run-time-table kernel (RSG_DECODE_NET=0), interleaved A B A B.
# Usage: bash tools/gpu_r4r.sh TAG
set -o pipefail
TAG=${1:-r4r}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -x -q --timeout 170 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 \
 && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
cd /tmp
for round in 1 2; do
  for net in 1 0; do
    for what in into2 heal; do
      RSG_DECODE_NET=$net EP_K=4 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/n${net}_${round}_$what -o run --output-format csv -- python3 $R/tools/engine_prof.py $what 10 > $OUT/n${net}_${round}_$what.txt 2>&1 || exit $?
    done
  done
done
echo done
