#!/bin/bash
# Round-end evidence, part A: full -m gpu suite, smoke, default bench (CPU
# baseline + extras), rocprof kernel stats of the default and --digests
# benches and of the one-pass GET / heal calls.  Each GPU step under its own
# time limit, chained with && (the first failure ends the call).
# Usage: bash tools/round_final.sh TAG
set -o pipefail
TAG=${1:-final}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
echo "host: $(hostname) nproc: $(nproc)" > $OUT/env.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1 \
 && tail -2 $OUT/pytest_gpu.log \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
 && timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err \
 && cd /tmp \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o bench --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $OUT/bench_under_rocprof.json 2> $OUT/prof.err \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_digests -o digests --output-format csv -- python3 $R/bench.py --digests --no-cpu-baseline > $OUT/digests_under_rocprof.json 2>> $OUT/prof.err \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_get2 -o get2 --output-format csv -- python3 $R/tools/engine_prof.py get2 20 > $OUT/get2.txt 2>> $OUT/prof.err \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_heal -o heal --output-format csv -- python3 $R/tools/engine_prof.py heal 20 > $OUT/heal.txt 2>> $OUT/prof.err \
 && echo done > $OUT/DONE
