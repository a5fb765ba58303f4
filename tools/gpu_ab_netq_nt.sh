#!/bin/bash
# Non-temporal 8-byte stores in the four-wave network kernels (B) against cached
# (A): RS(12,4) / RS(10,4) fused encode (tools/fused_kinds.py) and GET / heal
# (tools/geom_engines.py), A B A B.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab_netq_nt
mkdir -p $OUT
for i in 1 2; do
  for v in A B; do
    for g in "12 4" "10 4"; do
      RSG_LIB_PATH=$R/rustfs_amd/ab/$v.so timeout -k 10 120 python -u tools/fused_kinds.py $g auto >> $OUT/fused_$v$i.jsonl 2>> $OUT/err.txt || exit 1
    done
    RSG_LIB_PATH=$R/rustfs_amd/ab/$v.so timeout -k 10 200 python -u tools/geom_engines.py 12,4 10,4 > $OUT/geom_$v$i.jsonl 2>> $OUT/err.txt || exit 1
  done
done
echo done
