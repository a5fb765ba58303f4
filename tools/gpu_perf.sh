#!/bin/bash
# Perf pass on the GPU box: bench variants (each under its own time limit).
. "$(dirname "$0")/measure_env.sh"  # RSG_* knobs: the measurement build (ABI 6)
set -o pipefail
TAG=${1:-perf}
OUT=gpurun_out/$TAG
mkdir -p $OUT
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras"
timeout -k 10 300 $B > $OUT/encode.json 2>>$OUT/err.log \
 && timeout -k 10 300 $B --digests > $OUT/encode_hash_fused.json 2>>$OUT/err.log \
 && RSG_FUSED=0 timeout -k 10 300 $B --digests > $OUT/encode_hash_unfused.json 2>>$OUT/err.log \
 && timeout -k 10 300 $B --k 16 --m 4 > $OUT/encode_16_4.json 2>>$OUT/err.log
