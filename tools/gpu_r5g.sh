#!/bin/bash
# Round-5 pass G: the GPU suite and smoke with the EC:5..8 (m > 4) one-pass
# kernels (k_decode_records_dma with 8 row slots), one-pass / two-pass / AUTO
# GET and heal at those geometries (tools/geom_engines.py), and a rocprofv3
# kernel trace of RS(8,8)'s run naming the kernels that ran.
# Usage: bash tools/gpu_r5g.sh TAG
set -o pipefail
TAG=${1:-r5g}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 170 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 \
 && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 400 python -u tools/geom_engines.py 8,8 10,6 5,5 11,5 7,7 9,7 6,6 > $OUT/geom_engines.jsonl 2> $OUT/geom_engines.err || exit 1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof88 -o run -- python3 $R/tools/geom_engines.py 8,8 --reps 5 > $OUT/prof88.log 2>&1 || exit 1
echo done
