#!/bin/bash
# Round-4 pass E: RS(12,4) network kernels with four network waves (one per
# SIMD; every listed pattern, ragged walks, RS(16,4) / RS(8,4) network
# tests after the net16 clean-up), their kernel stats, the RS(12,4) line and
# the default line (engine kernel times now the median, with every call's).
# Usage: bash tools/gpu_r4e.sh TAG
set -o pipefail
TAG=${1:-r4e}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_decode_nets.py tests/test_gpu_decode.py -x -q --timeout 170 --timeout-method thread -m gpu -k "rs12 or rs16 or long or ragged or every_pattern" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
cd /tmp
for what in into2 heal into0; do
  EP_K=12 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/k12_$what -o run --output-format csv -- python3 $R/tools/engine_prof.py $what 10 > $OUT/k12_$what.txt 2>&1 || exit $?
done
cd $R
timeout -k 10 400 python -u bench.py --k 12 --m 4 --no-cpu-baseline --no-config-extras > $OUT/bench_12_4.json 2> $OUT/bench_12_4.err || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
echo done
