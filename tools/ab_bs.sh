#!/bin/bash
# Bit-sliced encode (k_encode_bs) against the v_perm table kernels: RS(16,4)
# (config 5: 1 MiB stripes, n = 8192) and RS(8,4) (the headline, n = 4096),
# encode only, one process per setting (knobs are read once per process).
# Output: gpurun_out/<TAG>/<geo>_<setting>.json
# Usage: bash tools/ab_bs.sh TAG
set -o pipefail
TAG=${1:-ab_bs}
OUT=gpurun_out/$TAG
mkdir -p $OUT
run() {  # geo name env... -- bench args
  local geo=$1 name=$2; shift 2
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 150 python bench.py "$@" --steps 20 --warmup 3 --no-extras --no-cpu-baseline \
      --no-config-extras > $OUT/${geo}_${name}.json 2> $OUT/${geo}_${name}.err || exit $?
  python - $OUT/${geo}_${name}.json $geo $name <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"]
print(f"{sys.argv[2]:5s} {sys.argv[3]:8s} kernel {r['kernel_ms_avg']:.4f} ms (min {r['kernel_ms_min']:.4f}) frac {r['frac']:.4f} value {d['value']:.2f}", flush=True)
PY
}
for rep in 1 2; do
  run rs164 table RSG_BITSLICE=0 -- --k 16 --m 4 --batch 8192
  run rs164 bs_nt3 RSG_BS_NT=3 -- --k 16 --m 4 --batch 8192
  run rs164 contig_nt1 RSG_BS_CONTIG=1 RSG_BS_NT=1 -- --k 16 --m 4 --batch 8192
  run rs164 contig_nt2 RSG_BS_CONTIG=1 RSG_BS_NT=2 -- --k 16 --m 4 --batch 8192
  run rs164 cseq3 RSG_BS_CONTIG=1 RSG_BS_SEQ=1 RSG_BS_OCC=3 -- --k 16 --m 4 --batch 8192
  run rs164 cseq3_nt2 RSG_BS_CONTIG=1 RSG_BS_SEQ=1 RSG_BS_OCC=3 RSG_BS_NT=2 -- --k 16 --m 4 --batch 8192
  run rs164 seq3_nt2 RSG_BS_SEQ=1 RSG_BS_OCC=3 RSG_BS_NT=2 -- --k 16 --m 4 --batch 8192
  run rs84 table RSG_BITSLICE=0 --
  run rs84 contig RSG_BITSLICE=1 RSG_BS_CONTIG=1 --
  run rs84 contig_nt1 RSG_BITSLICE=1 RSG_BS_CONTIG=1 RSG_BS_NT=1 --
  run rs84 contig_nt2 RSG_BITSLICE=1 RSG_BS_CONTIG=1 RSG_BS_NT=2 --
done
