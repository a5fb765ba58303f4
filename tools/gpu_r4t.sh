#!/bin/bash
# Round-4 pass T: the rebuilt library (comment-only source changes) — the
# whole GPU suite and smoke.  Usage: bash tools/gpu_r4t.sh TAG
set -o pipefail
TAG=${1:-r4t}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -x -q --timeout 170 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 \
 && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
tail -1 $OUT/smoke.log
