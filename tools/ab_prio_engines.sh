#!/bin/bash
# Wave-priority A/B of the one-pass engines (rsg_set_tuning RSG_DMA_PRIO:
# 0 none, 1 hash waves raised, 2 GF / network waves raised (default), 3 both)
# at RS(12,4), RS(8,4), RS(10,4) (networks) and RS(11,4) (table kernel),
# interleaved twice on one box.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab_prio_eng
mkdir -p $OUT
for i in 1 2; do
  for P in 2 0 1 3; do
    timeout -k 10 300 python -u tools/geom_engines.py 12,4 8,4 10,4 11,4 --tune RSG_DMA_PRIO=$P > $OUT/prio${P}_$i.jsonl 2>> $OUT/err.txt || exit 1
  done
done
echo done
