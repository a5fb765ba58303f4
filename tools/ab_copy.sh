#!/bin/bash
# A/B of the hash kernel's copy mode (RSG_HASH_COPY=1: direct 8-byte stores;
# default: LDS-staged 16-byte stores) on the GET engine, after the GPU tests.
. "$(dirname "$0")/measure_env.sh"  # RSG_* knobs: the measurement build (ABI 6)
set -o pipefail
TAG=${1:-abcopy}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
 && RSG_HASH_COPY=1 timeout -k 10 300 python tools/engine_bench.py > $OUT/engine_c1.json 2> $OUT/err1.log \
 && timeout -k 10 300 python tools/engine_bench.py > $OUT/engine_c2.json 2> $OUT/err2.log \
 && RSG_HASH_COPY=1 timeout -k 10 300 python tools/engine_bench.py > $OUT/engine_c1b.json 2>> $OUT/err1.log \
 && timeout -k 10 300 python tools/engine_bench.py > $OUT/engine_c2b.json 2>> $OUT/err2.log
