#!/bin/bash
# SQ counter passes over the one-pass GET / heal engine calls and the fused
# encode bench (kernel trace only, one counter group per pass).
# Usage: [WHATS="get2 heal"] [TRAFFIC=1] [NOFUSED=1] bash tools/pmc_engine.sh TAG
set -o pipefail
TAG=${1:-pmc_engine}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE"
G2="SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_COUNT"
G3="FETCH_SIZE"
G4="WRITE_SIZE"
for what in ${WHATS:-get2 heal}; do
  i=0
  for CTRS in "$G1" "$G2" ${TRAFFIC:+"$G3" "$G4"}; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTRS -d $OUT/$what/p$i -o run --output-format csv -- python3 $R/tools/engine_prof.py $what 3 > $OUT/${what}_p$i.txt 2>&1 || exit $?
  done
done
[ -n "$NOFUSED" ] && exit 0
i=0
for CTRS in "$G1" "$G2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTRS -d $OUT/fused/p$i -o run --output-format csv -- python3 $R/bench.py --digests --steps 3 --warmup 1 --no-extras --no-cpu-baseline > $OUT/fused_p$i.txt 2>&1 || exit $?
done
