#!/bin/bash
# HBM traffic of every kernel of the default bench line: FETCH_SIZE and
# WRITE_SIZE in passes of their own (kernel trace only) over one short
# default run; tools/pmc_bench_traffic.py turns them into the line's
# tools/pmc_traffic.json entries.  Usage: bash tools/pmc_bench.sh TAG
set -o pipefail
TAG=${1:-pmc_bench}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for CTRS in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $CTRS -d $OUT/p$i -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_p$i.json 2> $OUT/bench_p$i.err || exit $?
done
echo done
