#!/bin/bash
# PMC passes (one counter group per pass, --kernel-trace only; never combined
# with sys/runtime traces).  Usage: bash tools/pmc.sh TAG "bench args"
set -o pipefail
TAG=${1:-pmc}
ARGS=${2:-"--steps 3 --warmup 1 --no-extras --no-cpu-baseline"}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for CTRS in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE" "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $CTRS -d $OUT/p$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/bench_p$i.json 2> $OUT/err_p$i.log || exit $?
done
