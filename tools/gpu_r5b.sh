#!/bin/bash
# Round-5 pass B: the GPU suite (odd-k table-kernel patterns, RS(16,4) on the
# table kernel, async rotten records, slot aliasing, versioned loopback) and
# smoke on the rebuilt library (compressed code objects, no RS(16,4)
# networks), the default bench line, then one-pass against two-pass GET /
# heal at the geometries without a network (tools/geom_engines.py), and the
# PMC traffic table of every configuration the line prices (tools/pmc_table.sh).
# Each GPU step has its own time limit; && / exit end the call at the first
# failure.  Usage: bash tools/gpu_r5b.sh TAG
set -o pipefail
TAG=${1:-r5b}
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
timeout -k 10 400 python -u tools/geom_engines.py 5,4 11,4 15,1 9,4 13,3 7,1 3,2 16,4 12,4 10,4 > $OUT/geom_engines.jsonl 2> $OUT/geom_engines.err || exit 1
bash tools/pmc_table.sh $TAG/pmc > $OUT/pmc_table.log 2>&1 || { tail -20 $OUT/pmc_table.log; exit 1; }
echo done
