#!/bin/bash
# Round-3 evidence pass at HEAD: the default bench line (headline + config
# 3/4/5 extras + engines + CPU baseline), the same command under rocprofv3
# --kernel-trace --stats (its per-kernel averages must reproduce the line's
# kernel_ms), RS(16,4) engines (bench.py --k 16 --m 4), and the config-4 few
# large stripes at 4 GiB sizing.  Each GPU step has its own time limit; &&
# ends the call at the first failure.  Usage: bash tools/gpu_r3_final.sh TAG
set -o pipefail
TAG=${1:-r3_final}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "host: $(hostname) nproc: $(nproc)" > $OUT/env.txt
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err \
 && timeout -k 10 300 python -u bench.py --k 16 --m 4 --no-cpu-baseline --no-config-extras > $OUT/bench_16_4.json 2>> $OUT/bench.err \
 && cd /tmp \
 && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err \
 && cd $R \
 && bash tools/ab_fused_kind.sh $TAG/kind auto > $OUT/kind.txt 2>&1
rc=$?
cat $OUT/kind.txt 2>/dev/null
exit $rc
