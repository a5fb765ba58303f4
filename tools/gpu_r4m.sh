#!/bin/bash
# Round-4 pass M: the RS(12,4) fused encode + HH256S on a 2-slot ring with
# two workgroups per CU (the accumulators doubling as the target-row area)
# against the 4-slot one-workgroup form (RSG_NET12_RD=4): parity tests of both,
# then the --digests line's kernel stats interleaved A B A B.
# Usage: bash tools/gpu_r4m.sh TAG
set -o pipefail
TAG=${1:-r4m}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_decode_nets.py -x -q --timeout 170 --timeout-method thread -m gpu -k "fused or batch_encode or rs12 or knobs" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
RSG_NET12_RD=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 170 --timeout-method thread -m gpu -k "fused" > $OUT/pytest_rd4.log 2>&1 || { tail -40 $OUT/pytest_rd4.log; exit 1; }
tail -2 $OUT/pytest_rd4.log
cd /tmp
for round in 1 2; do
  for rd in 2 4; do
    RSG_NET12_RD=$rd timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/rd${rd}_${round}_fused12 -o run --output-format csv -- python3 $R/bench.py --k 12 --m 4 --digests --no-extras --no-cpu-baseline > $OUT/rd${rd}_${round}_fused12.json 2> $OUT/rd${rd}_${round}_fused12.err || exit $?
  done
done
echo done
