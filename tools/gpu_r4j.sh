#!/bin/bash
# Round-4 pass J: the record engines' verdict copy-back as a kernel on the
# call's stream (k_copy_to_host) instead of a copy-engine transfer: engine
# tests (sync, async, host-batch), the engine kernel stats and the default
# line (asynchronous GET / heal per-call time against the kernel time).
# Usage: bash tools/gpu_r4j.sh TAG
set -o pipefail
TAG=${1:-r4j}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_decode.py tests/test_gpu_heal.py tests/test_gpu_host_async.py tests/test_gpu_engine.py tests/test_gpu_decode_nets.py -x -q --timeout 170 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
cd /tmp
for what in into2 heal; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/k8_$what -o run --output-format csv -- python3 $R/tools/engine_prof.py $what 10 > $OUT/k8_$what.txt 2>&1 || exit $?
done
cd $R
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
echo done
