#!/bin/bash
# Round-4 pass F: RS(12,4) network kernels with LDS-atomic row accumulators
# and a 4-slot ring, and the RS(12,4) fused encode + HH256S as the network
# heal of every parity shard (k_encode_hash_net12): parity tests, kernel
# stats, the RS(12,4) lines (plain and --digests) and the default line.
# Usage: bash tools/gpu_r4f.sh TAG
set -o pipefail
TAG=${1:-r4f}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_decode_nets.py tests/test_gpu_decode.py tests/test_gpu_parity.py -x -q --timeout 170 --timeout-method thread -m gpu -k "rs12 or rs16 or long or ragged or every_pattern or fused or batch_encode" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
cd /tmp
for what in into2 heal; do
  EP_K=12 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/k12_$what -o run --output-format csv -- python3 $R/tools/engine_prof.py $what 10 > $OUT/k12_$what.txt 2>&1 || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/fused12 -o run --output-format csv -- python3 $R/bench.py --k 12 --m 4 --digests --no-extras --no-cpu-baseline > $OUT/bench_12_4_digests.json 2> $OUT/fused12.err || exit $?
cd $R
timeout -k 10 400 python -u bench.py --k 12 --m 4 --no-cpu-baseline --no-config-extras > $OUT/bench_12_4.json 2> $OUT/bench_12_4.err || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
echo done
