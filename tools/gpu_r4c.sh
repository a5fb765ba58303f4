#!/bin/bash
# Round-4 pass C: RS(12,4) one-pass GET/heal with the 4-slot ring
# (correctness on every listed pattern, then rocprof kernel stats), the fused
# encode + HH256S at RS(12,4) (packed kernel, ragged chunks), and an A/B of
# the RS(12,4) encode kernel's launch shape (RSG_VEC_BLOCK / RSG_VEC_OCC).
# Usage: bash tools/gpu_r4c.sh TAG
set -o pipefail
TAG=${1:-r4c}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode_nets.py -x -q --timeout 170 --timeout-method thread -m gpu -k "rs12 or long" > $OUT/pytest_rs12.log 2>&1 || { tail -40 $OUT/pytest_rs12.log; exit 1; }
tail -2 $OUT/pytest_rs12.log
cd /tmp
for what in into2 heal into0; do
  EP_K=12 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/k12_$what -o run --output-format csv -- python3 $R/tools/engine_prof.py $what 10 > $OUT/k12_$what.txt 2>&1 || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/fused12 -o run --output-format csv -- python3 $R/bench.py --k 12 --m 4 --digests --no-extras --no-cpu-baseline > $OUT/bench_12_4_digests.json 2> $OUT/fused12.err || exit $?
cd $R
for env in "X=1" "RSG_VEC_BLOCK=256" "RSG_VEC_OCC=2" "RSG_VEC_OCC=3" "RSG_VEC_OCC=4" "RSG_VEC_BLOCK=256 RSG_VEC_OCC=2"; do
  echo "== $env" >> $OUT/enc12_ab.txt
  env $env timeout -k 10 120 python bench.py --k 12 --m 4 --no-extras --no-cpu-baseline --steps 30 >> $OUT/enc12_ab.txt 2>&1 || exit $?
done
echo done
