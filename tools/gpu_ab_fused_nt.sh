#!/bin/bash
# Non-temporal parity stores in the packed and ring fused kernels (B) against
# plain stores (A): the fused tests on B, then tools/fused_kinds.py A B twice.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab_fused_nt
mkdir -p $OUT
RSG_LIB_PATH=$R/rustfs_amd/ab/B.so timeout -k 10 300 python -u -m pytest tests -x -q --timeout 60 --timeout-method thread -m gpu -k "fused" > $OUT/pytest_B.log 2>&1 || { tail -20 $OUT/pytest_B.log; exit 1; }
tail -1 $OUT/pytest_B.log
for i in 1 2; do
  for v in A B; do
    for g in "5 4 auto" "3 2 auto" "7 1 auto" "2 2 auto" "8 4 ring packed"; do
      RSG_LIB_PATH=$R/rustfs_amd/ab/$v.so timeout -k 10 120 python -u tools/fused_kinds.py $g >> $OUT/$v$i.jsonl 2>> $OUT/err.txt || exit 1
    done
  done
done
echo done
