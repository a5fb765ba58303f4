#!/bin/bash
# BASELINE config 4: RS(8,4) encode + fused HH256S digests over a 64 KiB-16 MiB
# stripe sweep (and the same sweep without digests for reference), one GPU.
# Batch: at least 4096 stripes, at least ~6 GiB of stripes per launch.
# Output: gpurun_out/<TAG>/*.json (one bench.py line each); summarise with
#   python tools/sweep_summary.py gpurun_out/<TAG> > profiles/rNN/sweep_fused.md
# Usage: bash tools/sweep_fused.sh [TAG]  (default: sweep)
set -eo pipefail
cd "$(dirname "$0")/.."
TAG=${1:-sweep}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for kib in 64 128 256 512 1024 2048 4096 8192 16384; do
    bytes=$((kib * 1024))
    n=$(( (6 * 1024 * 1024 * 1024) / (bytes * 3 / 2) ))
    [ "$n" -lt 4096 ] && n=4096
    for mode in hash plain; do
        flag=""
        [ "$mode" = hash ] && flag="--digests"
        echo "stripe ${kib} KiB n=${n} ${mode}"
        timeout -k 10 300 python bench.py --stripe-bytes "$bytes" --batch "$n" $flag --steps 10 --warmup 2 \
            --no-extras --no-cpu-baseline --no-config-extras > "$OUT/s${kib}k_${mode}.json"
        tail -1 "$OUT/s${kib}k_${mode}.json" | cut -c1-160
    done
    # SURVEY §8(d) config 4 sizing: n * stripe = 4 GiB (fewer than 4096 stripes above 1 MiB)
    n4=$(( (4 * 1024 * 1024 * 1024) / bytes ))
    if [ "$n4" -lt 4096 ]; then
        echo "stripe ${kib} KiB n=${n4} hash (4 GiB payload)"
        timeout -k 10 300 python bench.py --stripe-bytes "$bytes" --batch "$n4" --digests --steps 10 --warmup 2 \
            --no-extras --no-cpu-baseline --no-config-extras > "$OUT/s${kib}k_hash4g.json"
        tail -1 "$OUT/s${kib}k_hash4g.json" | cut -c1-160
    fi
done
