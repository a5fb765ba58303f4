#!/bin/bash
# SQ counters of the bit-sliced encode against the table kernels (RS(8,4)
# n = 4096, RS(16,4) n = 8192), one counter group per pass, kernel trace only.
# Usage: bash tools/pmc_bs.sh TAG
set -o pipefail
TAG=${1:-pmc_bs}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE"
G2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_INSTS_SALU GRBM_COUNT"
B="--steps 3 --warmup 1 --no-extras --no-cpu-baseline --no-config-extras"
for what in "rs84_table RSG_BITSLICE=0 --" "rs84_bs RSG_BITSLICE=1 RSG_BS_NT=3 --" \
            "rs164_table RSG_BITSLICE=0 -- --k 16 --m 4 --batch 8192" \
            "rs164_seq3 RSG_BS_SEQ=1 RSG_BS_OCC=3 RSG_BS_NT=3 -- --k 16 --m 4 --batch 8192"; do
  set -- $what
  name=$1; shift
  envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  i=0
  for CTRS in "$G1" "$G2"; do
    i=$((i+1))
    export "${envs[@]}"
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTRS -d $OUT/$name/p$i -o run --output-format csv -- python3 $R/bench.py $B "$@" > $OUT/${name}_p$i.txt 2>&1 || exit $?
    unset RSG_BITSLICE RSG_BS_NT RSG_BS_SEQ RSG_BS_OCC
  done
  python3 $R/tools/pmc_summary.py $OUT/$name "rsg::k_" > $OUT/${name}_summary.txt
done
