#!/bin/bash
# A/B of the hash kernel's prefetch depth (RSG_HASH_DEEP) on the engines that
# are hash-bound (GET verify+gather, bitrot_verify, heal), after the GPU tests.
set -o pipefail
TAG=${1:-abhash}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
 && RSG_HASH_DEEP=0 timeout -k 10 300 python tools/engine_bench.py > $OUT/engine_d0.json 2> $OUT/err0.log \
 && RSG_HASH_DEEP=1 timeout -k 10 300 python tools/engine_bench.py > $OUT/engine_d1.json 2> $OUT/err1.log \
 && RSG_HASH_DEEP=0 timeout -k 10 300 python tools/engine_bench.py > $OUT/engine_d0b.json 2>> $OUT/err0.log \
 && RSG_HASH_DEEP=1 timeout -k 10 300 python tools/engine_bench.py > $OUT/engine_d1b.json 2>> $OUT/err1.log
