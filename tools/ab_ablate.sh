#!/bin/bash
# Ablation of the network GET/heal kernel: kernel times (rocprofv3 kernel
# stats over tools/engine_prof.py, which checks nothing) of the production
# library and of exp/librsgpu_ablate.so (built with -DRSG_NET_ABLATE=1: the
# network waves load, store and compare but do no transposes or XORs).
# Usage: bash tools/ab_ablate.sh TAG
. "$(dirname "$0")/measure_env.sh"  # RSG_* knobs: the measurement build (ABI 6)
set -o pipefail
TAG=${1:-r3_ablate}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for lib in prod ablate; do
  for what in heal get2; do
    if [ $lib = ablate ]; then export RSG_LIB_PATH=$R/exp/librsgpu_ablate.so; else unset RSG_LIB_PATH; fi
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/${lib}_$what -o run --output-format csv -- python3 $R/tools/engine_prof.py $what 8 > $OUT/${lib}_$what.txt 2>&1 || exit $?
    f=$(find $OUT/${lib}_$what -name 'run_kernel_stats.csv' | head -1)
    grep records_net $f | cut -d, -f1-4 | sed "s/^/$lib $what /"
  done
done
