#!/bin/bash
# One GPU-box pass: build check, parity tests, smoke, bench, rocprof kernel stats.
# Every GPU step has its own time limit; steps are chained with && so the first
# failure ends the call.  Usage (from the repo root, via gpurun):
#   bash tools/gpu_check.sh [tag]
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "host: $(hostname) cpus: $(nproc)" > $OUT/env.txt
rocm-smi --showproductname >> $OUT/env.txt 2>&1 || true
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $OUT/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
 && timeout -k 10 600 python bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err \
 && cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/bench_prof.json 2> $GRAFT_REPO_ROOT/$OUT/prof.err
rc=$?
echo "exit $rc" >> $GRAFT_REPO_ROOT/$OUT/env.txt
exit $rc
