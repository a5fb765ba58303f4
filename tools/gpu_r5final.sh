#!/bin/bash
# Round-5 final pass on the shipped library: the GPU suite and smoke, the
# default bench line, the same line under rocprofv3 --kernel-trace --stats
# (per-kernel summary for profiles/), and one-pass / two-pass / AUTO GET and
# heal at the geometries without networks (tools/geom_engines.py).  The PMC
# traffic table is a second call (tools/pmc_table.sh).  Each GPU step has its
# own time limit; the first failure ends the call.
# Usage: bash tools/gpu_r5final.sh TAG
set -o pipefail
TAG=${1:-r5final}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "host: $(hostname)" > $OUT/env.txt
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 \
 && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py > $OUT/bench_prof.json 2> $OUT/bench_prof.err || exit 1
cd $R && timeout -k 10 500 python -u tools/geom_engines.py 5,4 11,4 15,1 9,4 13,3 7,1 3,2 14,2 8,8 10,6 > $OUT/geom_engines.jsonl 2> $OUT/geom_engines.err && timeout -k 10 300 python -u tools/verify_geoms.py 12,4 10,4 6,4 5,4 3,2 14,2 8,4 > $OUT/verify_geoms.jsonl 2> $OUT/verify_geoms.err || exit 1
echo done
