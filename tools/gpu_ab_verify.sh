#!/bin/bash
# The DMA-ring verify (B, rs_verify.hip) against the quad kernel (A) for
# records at unaligned pitches: the GPU suite on B, then tools/verify_geoms.py
# on A and B interleaved twice.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab_verify
mkdir -p $OUT
RSG_LIB_PATH=$R/rustfs_amd/ab/B.so timeout -k 10 600 python -u -m pytest tests -x -q --timeout 60 --timeout-method thread -m gpu > $OUT/pytest_gpu_B.log 2>&1 || { tail -30 $OUT/pytest_gpu_B.log; exit 1; }
tail -1 $OUT/pytest_gpu_B.log
for i in 1 2; do
  for v in A B; do
    RSG_LIB_PATH=$R/rustfs_amd/ab/$v.so timeout -k 10 300 python -u tools/verify_geoms.py 12,4 10,4 6,4 14,2 5,4 3,2 8,4 > $OUT/$v$i.jsonl 2>> $OUT/err.txt || exit 1
  done
done
echo done
