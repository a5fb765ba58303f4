#!/bin/bash
# Round-4 pass H: HBM traffic (FETCH_SIZE / WRITE_SIZE, one counter per
# pass, kernel trace only) and VALU instruction counts for the RS(12,4)
# lines and engines and the RS(8,4) heal, for tools/pmc_traffic.json and
# DESIGN.md.  Usage: bash tools/gpu_r4h.sh TAG
set -o pipefail
TAG=${1:-r4h}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for CTRS in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTRS -d $OUT/enc12/p$i -o run --output-format csv -- python3 $R/bench.py --k 12 --m 4 --steps 3 --warmup 1 --no-extras --no-cpu-baseline > $OUT/enc12_p$i.txt 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTRS -d $OUT/fused12/p$i -o run --output-format csv -- python3 $R/bench.py --k 12 --m 4 --digests --steps 3 --warmup 1 --no-extras --no-cpu-baseline > $OUT/fused12_p$i.txt 2>&1 || exit $?
  for what in into2 heal into0; do
    EP_K=12 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTRS -d $OUT/k12_$what/p$i -o run --output-format csv -- python3 $R/tools/engine_prof.py $what 3 > $OUT/k12_${what}_p$i.txt 2>&1 || exit $?
  done
  EP_K=8 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTRS -d $OUT/k8_heal/p$i -o run --output-format csv -- python3 $R/tools/engine_prof.py heal 3 > $OUT/k8_heal_p$i.txt 2>&1 || exit $?
done
cd $R
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
echo done
