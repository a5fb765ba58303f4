#!/bin/bash
# Round-4 pass N: the other default geometries of rustfs's erasure sets
# (storageclass.rs:24-31: 8 drives RS(4,4), 10 drives RS(6,4), 14 drives
# RS(10,4)) at 1 MiB blocks, n = 4096: GET in place with 2 data lost, GET with
# all present, heal of a data + a parity disk (kernel stats), and the encode
# and encode + fused HH256S lines.  Usage: bash tools/gpu_r4n.sh TAG
set -o pipefail
TAG=${1:-r4n}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for k in 4 6 10; do
  cd /tmp
  for what in into2 into0 heal; do
    EP_K=$k timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/k${k}_$what -o run --output-format csv -- python3 $R/tools/engine_prof.py $what 10 > $OUT/k${k}_$what.txt 2>&1 || exit $?
  done
  cd $R
  timeout -k 10 300 python -u bench.py --k $k --m 4 --no-extras --no-cpu-baseline > $OUT/bench_k$k.json 2> $OUT/bench_k$k.err || exit 1
  timeout -k 10 300 python -u bench.py --k $k --m 4 --digests --no-extras --no-cpu-baseline > $OUT/bench_k${k}_digests.json 2> $OUT/bench_k${k}_digests.err || exit 1
done
echo done
