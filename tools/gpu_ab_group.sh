#!/bin/bash
# A/B: the table kernel's 8-stripe workgroups for <= 8 survivors (A) against
# 4-stripe workgroups for every survivor count (B, RSG_GET_GROUP_SMALL=4):
# tools/geom_engines.py on both, A B A B; RS(8,4)/RS(6,4)/RS(4,4) with the
# networks off so the table kernel runs.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab_group
mkdir -p $OUT
for i in 1 2; do
  for v in A B; do
    RSG_LIB_PATH=$R/rustfs_amd/ab/$v.so timeout -k 10 300 python -u tools/geom_engines.py 5,4 3,2 7,1 2,2 > $OUT/geom_$v$i.jsonl 2>> $OUT/err.txt || exit 1
    RSG_LIB_PATH=$R/rustfs_amd/ab/$v.so timeout -k 10 300 python -u tools/geom_engines.py 8,4 6,4 4,4 --tune RSG_DECODE_NET=0 > $OUT/geomtab_$v$i.jsonl 2>> $OUT/err.txt || exit 1
  done
done
echo done
