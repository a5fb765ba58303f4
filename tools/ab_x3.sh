#!/bin/bash
# A/B after a kernel change: GPU parity tests, then ring/packed microbench and
# the config-2/4/5 bench lines.  Each GPU step has its own time limit.
set -o pipefail
TAG=${1:-ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
 && timeout -k 10 120 tools/kbench/ring_variants 2097152 256 6 > $OUT/ring_s16m.txt 2>&1 \
 && timeout -k 10 120 tools/kbench/ring_variants 131072 4096 6 > $OUT/ring_s1m.txt 2>&1 \
 && timeout -k 10 300 $B > $OUT/encode.json 2>>$OUT/err.log \
 && timeout -k 10 300 $B --digests > $OUT/encode_hash.json 2>>$OUT/err.log \
 && timeout -k 10 300 $B --k 16 --m 4 > $OUT/encode_16_4.json 2>>$OUT/err.log
