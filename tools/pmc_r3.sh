#!/bin/bash
# Round-3 PMC traffic / issue passes: config 5's per-GPU RS(16,4) encode and
# config 4's wide-kernel points (4 and 8 MiB stripes at 4 GiB sizing).
set -o pipefail
B="--steps 3 --warmup 1 --warm-seconds 0 --no-extras --no-cpu-baseline --no-config-extras"
bash tools/pmc.sh r3_pmc_rs164 "--k 16 --m 4 --batch 8192 $B" \
 && bash tools/pmc.sh r3_pmc_w4 "--stripe-bytes 4194304 --batch 1024 --digests $B" \
 && bash tools/pmc.sh r3_pmc_w8 "--stripe-bytes 8388608 --batch 512 --digests $B"
