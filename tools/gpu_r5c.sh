#!/bin/bash
# Round-5 pass C: the GPU suite and smoke on the library with the k*R table
# policy, the default bench line, its rocprofv3 kernel-trace --stats run (the
# per-kernel averages must agree with the line), the geometry A/B of the
# policy's edges, and the PMC traffic table (tools/pmc_table.sh).
# Usage: bash tools/gpu_r5c.sh TAG
set -o pipefail
TAG=${1:-r5c}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "host: $(hostname) nproc: $(nproc)" > $OUT/env.txt
timeout -k 10 500 python -u -m pytest tests -x -q --timeout 170 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 \
 && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
cd $R
timeout -k 10 300 python -u tools/geom_engines.py 11,4 13,3 16,4 9,4 > $OUT/geom_engines.jsonl 2> $OUT/geom_engines.err || exit 1
bash tools/pmc_table.sh $TAG/pmc > $OUT/pmc_table.log 2>&1 || { tail -20 $OUT/pmc_table.log; exit 1; }
echo done
