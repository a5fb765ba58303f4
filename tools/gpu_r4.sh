#!/bin/bash
# Round-4 GPU pass: parity suite, smoke, the default bench line (headline +
# config 3/4/5 extras + engines + CPU baseline), and a rocprof kernel-stats run
# of the same default command whose per-kernel averages must agree with the
# line's kernel_ms.  Each GPU step has its own time limit; && ends the call
# at the first failure.  Usage: bash tools/gpu_r4.sh TAG [skip-tests|tests] [no-prof]
set -o pipefail
TAG=${1:-r4}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "host: $(hostname) nproc: $(nproc)" > $OUT/env.txt
run_tests() {
  timeout -k 10 600 python -u -m pytest tests -x -q --timeout 170 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 \
  && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
}
if [ "$2" != "skip-tests" ]; then run_tests || { tail -30 $OUT/pytest_gpu.log; exit 1; }; fi
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err \
 && { [ "$3" = "no-prof" ] || { cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/bench_prof.json 2> $GRAFT_REPO_ROOT/$OUT/prof.err; }; }
rc=$?
cd $GRAFT_REPO_ROOT
tail -3 $OUT/pytest_gpu.log 2>/dev/null
cat $OUT/bench.json
exit $rc
