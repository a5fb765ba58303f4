#!/bin/bash
# Round-4 pass I: A/B of the hash waves' record bases read once (current
# librsgpu.so) against re-read every step (librsgpu_prehoist.so, the same
# tree with that change undone), interleaved A B A B so the GPU's power
# state after sustained load weighs on both alike; then the default line.
# Usage: bash tools/gpu_r4i.sh TAG
set -o pipefail
TAG=${1:-r4i}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cp $R/rustfs_amd/librsgpu.so $R/rustfs_amd/librsgpu_hoist.so
cd /tmp
for round in 1 2; do
  for v in hoist prehoist; do
    cp $R/rustfs_amd/librsgpu_$v.so $R/rustfs_amd/librsgpu.so
    for kw in "12 into2" "12 heal" "8 into2" "8 heal"; do
      set -- $kw
      EP_K=$1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/${v}_${round}_k$1_$2 -o run --output-format csv -- python3 $R/tools/engine_prof.py $2 10 > $OUT/${v}_${round}_k$1_$2.txt 2>&1 || exit $?
    done
  done
done
cp $R/rustfs_amd/librsgpu_hoist.so $R/rustfs_amd/librsgpu.so
cd $R
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
echo done
