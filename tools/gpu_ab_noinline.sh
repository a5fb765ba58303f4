#!/bin/bash
# A/B of the record waves inlined into every kernel (A) against one noinline
# copy per shape reading the kernarg segment (B): the GPU suite on B, then
# bench.py interleaved A B A B A B, then the table-kernel geometries on both.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab_noinline
mkdir -p $OUT
export TMPDIR=/tmp
RSG_LIB_PATH=$R/rustfs_amd/ab/B.so timeout -k 10 600 python -u -m pytest tests -x -q --timeout 60 --timeout-method thread -m gpu > $OUT/pytest_gpu_B.log 2>&1 || { tail -30 $OUT/pytest_gpu_B.log; exit 1; }
tail -2 $OUT/pytest_gpu_B.log
bash tools/ab_libs.sh ab_noinline "--no-cpu-baseline" || exit 1
for v in A B; do
  RSG_LIB_PATH=$R/rustfs_amd/ab/$v.so timeout -k 10 300 python -u tools/geom_engines.py 11,4 13,3 5,4 8,8 10,4 14,2 9,4 > $OUT/geom_$v.jsonl 2> $OUT/geom_$v.err || exit 1
done
echo done
