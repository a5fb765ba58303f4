#!/bin/bash
# Round-5 pass A: the GPU suite and smoke on the rebuilt library, the default
# bench line, then the per-dispatch clock table of the one-pass engines —
# RS(8,4) heal (1 data + 1 parity) and in-place GET (2 data lost), 3 loops of
# 10 synchronous calls each after 0.5 s idle (round 4's engine protocol):
#   kt/  kernel trace alone (durations);
#   pmc/ GRBM_GUI_ACTIVE + GRBM_COUNT per dispatch beside the durations
#        (effective clock = GRBM_GUI_ACTIVE / 8 XCDs / duration).
# Each GPU step has its own time limit; && / exit end the call at the first
# failure.  Usage: bash tools/gpu_r5a.sh TAG
set -o pipefail
TAG=${1:-r5a}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "host: $(hostname) nproc: $(nproc)" > $OUT/env.txt
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 170 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 \
 && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
cd /tmp
for what in heal into2; do
  EP_LOOPS=3 EP_SLEEP=0.5 timeout -k 10 120 rocprofv3 --kernel-trace -d $OUT/kt_$what -o run --output-format csv \
    -- python3 $R/tools/engine_prof.py $what 10 > $OUT/kt_$what.txt 2>&1 || exit 1
  EP_LOOPS=3 EP_SLEEP=0.5 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/pmc_$what \
    -o run --output-format csv -- python3 $R/tools/engine_prof.py $what 10 > $OUT/pmc_$what.txt 2>&1 || exit 1
done
echo done
