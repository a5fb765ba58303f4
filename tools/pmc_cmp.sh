#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the GET GF pass in the engine (engine_prof.py
# get2_01) and in tools/kbench/get_probe, one counter per pass.
# Usage: bash tools/pmc_cmp.sh TAG
set -o pipefail
TAG=${1:-pmccmp}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d $OUT/eng_$C -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/engine_prof.py get2_01 3 > $OUT/eng_$C.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d $OUT/probe_$C -o run --output-format csv -- $GRAFT_REPO_ROOT/tools/kbench/get_probe 4096 1 0 0 0 > $OUT/probe_$C.log 2>&1 || exit $?
done
