#!/bin/bash
# Round-4 GPU pass B: the unaligned LDS-DMA probe gates everything after it
# (the one-pass kernels DMA records at any alignment); then the GPU suite,
# smoke, the default bench line and the RS(12,4) line, rocprof kernel stats
# of the RS(8,4) and RS(12,4) engine calls.
# Usage: bash tools/gpu_r4b.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-r4b}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 $R/tools/kbench/lds_dma_unaligned > $OUT/lds_unaligned.txt 2>&1 || exit 1
cat $OUT/lds_unaligned.txt
if grep -q WRONG $OUT/lds_unaligned.txt; then echo "unaligned LDS-DMA is not exact: stopping"; exit 3; fi
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q --timeout 170 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
fi
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
timeout -k 10 400 python -u bench.py --k 12 --m 4 --no-cpu-baseline --no-config-extras > $OUT/bench_12_4.json 2> $OUT/bench_12_4.err || { tail $OUT/bench_12_4.err; exit 1; }
cd /tmp
for k in 8 12; do
  for what in into0 into2 heal; do
    EP_K=$k timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/k${k}_$what -o run --output-format csv -- python3 $R/tools/engine_prof.py $what 10 > $OUT/k${k}_$what.txt 2>&1 || exit $?
  done
done
echo done
