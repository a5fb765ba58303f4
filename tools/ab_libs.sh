#!/bin/bash
# Interleaved A/B of two builds of the library on one box (RSG_LIB_PATH):
# rustfs_amd/ab/A.so and B.so, bench.py with the given arguments, A B A B A B.
# Usage: bash tools/ab_libs.sh TAG "bench args"
set -o pipefail
TAG=${1:-ab_libs}
ARGS=${2:-"--k 12 --m 4 --no-extras --no-cpu-baseline"}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
for i in 1 2 3; do
  for v in A B; do
    RSG_LIB_PATH=$R/rustfs_amd/ab/$v.so timeout -k 10 120 python -u bench.py $ARGS > $OUT/${v}$i.json 2> $OUT/${v}$i.err || exit 1
    python -c "import json,sys; d=json.loads(open('$OUT/${v}$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v$i', r['kernel_ms_avg'], r['frac'])"
  done
done
