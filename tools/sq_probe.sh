#!/bin/bash
# SQ counters of one bench-line configuration (tools/pmc_driver.py KEY): one
# rocprofv3 --pmc pass with up to 8 SQ counters, --kernel-trace only.
# Usage: bash tools/sq_probe.sh TAG KEY "COUNTERS"
set -o pipefail
TAG=$1; KEY=$2; CTRS=$3
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG/$KEY
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTRS -d $OUT/sq -o run --output-format csv \
  -- python3 $R/tools/pmc_driver.py $KEY $OUT 3 > $OUT/sq.log 2>&1 || { tail -5 $OUT/sq.log; exit 1; }
echo ok
