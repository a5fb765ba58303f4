#!/bin/bash
# Round-4 engine evidence: rocprof kernel stats of the GET (in-place and
# gather forms) and heal engine calls, and the PMC traffic passes
# (FETCH_SIZE, WRITE_SIZE: one counter per pass, kernel trace only) that
# tools/pmc_traffic.json is built from.  Usage: bash tools/gpu_eng_r4.sh TAG [tests]
set -o pipefail
TAG=${1:-eng_r4}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" = "tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q --timeout 170 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
cd /tmp
for what in ${WHATS:-into0 into2 get0 get2 heal}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/stats_$what -o run --output-format csv -- python3 $R/tools/engine_prof.py $what 10 > $OUT/stats_$what.txt 2>&1 || exit $?
  i=0
  for CTRS in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTRS -d $OUT/pmc_$what/p$i -o run --output-format csv -- python3 $R/tools/engine_prof.py $what 3 > $OUT/pmc_${what}_p$i.txt 2>&1 || exit $?
  done
done
echo done
