#!/bin/bash
# Round-4 pass G: wave-priority A/B (RSG_DMA_PRIO = 0 none, 1 hash waves,
# 2 GF/network waves (default), 3 both) of the one-pass kernels after the
# hash waves' record bases moved out of the step loop: RS(12,4) GET with 2
# data lost and heal, the RS(12,4) fused encode + HH256S, and the RS(8,4)
# GET; then the parity tests of the touched kernels.
# Usage: bash tools/gpu_r4g.sh TAG
set -o pipefail
TAG=${1:-r4g}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode_nets.py tests/test_gpu_parity.py tests/test_gpu_async.py tests/test_gpu_decode.py tests/test_gpu_heal.py -x -q --timeout 170 --timeout-method thread -m gpu -k "rs12 or long or ragged or fused or async or into or heal" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
cd /tmp
for prio in 0 1 2 3; do
  for what in into2 heal; do
    RSG_DMA_PRIO=$prio EP_K=12 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/p${prio}_k12_$what -o run --output-format csv -- python3 $R/tools/engine_prof.py $what 10 > $OUT/p${prio}_k12_$what.txt 2>&1 || exit $?
  done
  RSG_DMA_PRIO=$prio EP_K=8 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/p${prio}_k8_into2 -o run --output-format csv -- python3 $R/tools/engine_prof.py into2 10 > $OUT/p${prio}_k8_into2.txt 2>&1 || exit $?
  RSG_DMA_PRIO=$prio timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/p${prio}_fused12 -o run --output-format csv -- python3 $R/bench.py --k 12 --m 4 --digests --no-extras --no-cpu-baseline > $OUT/p${prio}_fused12.json 2> $OUT/p${prio}_fused12.err || exit $?
done
cd $R
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
echo done
