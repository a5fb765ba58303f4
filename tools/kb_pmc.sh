#!/bin/bash
# PMC passes over one tools/kbench binary (one counter group per pass, kernel
# trace only).  Usage: bash tools/kb_pmc.sh TAG BINARY [args...]
set -o pipefail
TAG=$1; BIN=$2; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for CTRS in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE" "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTRS -d $OUT/p$i -o run --output-format csv -- $GRAFT_REPO_ROOT/tools/kbench/$BIN "$@" > $OUT/out_p$i.txt 2>&1 || exit $?
done
