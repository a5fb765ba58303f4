#!/bin/bash
# GPU parity suite on the box: one pytest process, per-test timeout, log under
# gpurun_out/<tag>/.  Usage: bash tools/gpu_tests.sh TAG [pytest selectors...]
set -o pipefail
TAG=${1:-tests}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "host: $(hostname) nproc: $(nproc)" > $OUT/env.txt
timeout -k 10 1000 python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu "${@:-tests}" > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -5 $OUT/pytest_gpu.log
exit $rc
