#!/bin/bash
# Round-end evidence on one GPU: PMC traffic passes (encode, fused), rocprof
# kernel stats of the default bench and of the --digests bench, and the
# default bench line.  Every step under its own time limit; stops at the
# first failure.  Usage: bash tools/round_artifacts.sh TAG
set -o pipefail
TAG=${1:-r02}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/art_$TAG
mkdir -p $OUT
bash $R/tools/pmc.sh art_$TAG/pmc_enc "--steps 3 --warmup 1 --no-extras --no-cpu-baseline" || exit $?
bash $R/tools/pmc.sh art_$TAG/pmc_fused "--digests --steps 3 --warmup 1 --no-extras --no-cpu-baseline" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o bench --output-format csv -- python3 $R/bench.py > $OUT/bench_under_rocprof.json 2> $OUT/bench_under_rocprof.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_fused -o fused --output-format csv -- python3 $R/bench.py --digests --no-cpu-baseline > $OUT/fused_under_rocprof.json 2> $OUT/fused_under_rocprof.err || exit $?
timeout -k 10 300 python3 $R/bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit $?
echo done > $OUT/DONE
