#!/bin/bash
# Round-5 pass E: the GPU suite and smoke on the library whose table kernel
# runs 4-stripe workgroups of <= 8 waves on a 2-slot ring (two a CU), heals
# hashing their targets in the last hash wave, with the AUTO policy asking
# the launch shape; then one-pass / two-pass / AUTO GET and heal at the
# geometries that policy moves (tools/geom_engines.py); the default bench
# line before that.
# Usage: bash tools/gpu_r5e.sh TAG
set -o pipefail
TAG=${1:-r5e}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 170 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 \
 && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 400 python -u tools/geom_engines.py 11,4 13,3 14,4 9,4 15,4 16,4 14,2 > $OUT/geom_engines.jsonl 2> $OUT/geom_engines.err || exit 1
echo done
