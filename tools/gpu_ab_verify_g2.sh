#!/bin/bash
# Verify rings past 12 files: A (shipped: 13-15 files at even pitches on a
# 2-slot ring of 4 records a file, else the quad kernel), B (the same source
# rebuilt, control), C (RSG_VERIFY_G2=1: 13-16 files, any pitch, on a 3-slot
# ring of 2 records a file).  The GPU suite on C, then tools/verify_geoms.py
# A B C twice.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab_verify_g2
mkdir -p $OUT
RSG_LIB_PATH=$R/rustfs_amd/ab/C.so timeout -k 10 600 python -u -m pytest tests -x -q --timeout 60 --timeout-method thread -m gpu -k "verify or into or fullsize or decode" > $OUT/pytest_gpu_C.log 2>&1 || { tail -30 $OUT/pytest_gpu_C.log; exit 1; }
tail -1 $OUT/pytest_gpu_C.log
for i in 1 2; do
  for v in A B C; do
    RSG_LIB_PATH=$R/rustfs_amd/ab/$v.so timeout -k 10 300 python -u tools/verify_geoms.py 12,4 10,4 14,2 9,4 11,4 13,3 > $OUT/$v$i.jsonl 2>> $OUT/err.txt || exit 1
  done
done
echo done
