#!/bin/bash
# PMC traffic of every configuration bench.py's line prices (its `traffic`
# fields), on the shipped library: per key two rocprofv3 passes of
# tools/pmc_driver.py (FETCH_SIZE, then WRITE_SIZE; --kernel-trace only, one
# counter per pass), raw run_counter_collection.csv kept per key; then
# tools/pmc_traffic.py --from profiles/r05/pmc rebuilds tools/pmc_traffic.json
# (CPU side, after copying the outputs into profiles/).
# Usage: bash tools/pmc_table.sh TAG [keys...]
set -o pipefail
TAG=${1:-pmc_table}
shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
KEYS=${@:-"rs84_S131072_n4096 rs84_S131072_n4096_hash rs164_S65536_n4096 rs124_S87382_n4096 rs124_S87382_n4096_hash reconstruct_e1_rs84_S131072_n4096 reconstruct_e2_rs84_S131072_n4096 reconstruct_e3_rs84_S131072_n4096 reconstruct_e4_rs84_S131072_n4096 get_into0_rs84_S131072_n4096 get_into2_rs84_S131072_n4096 heal_1d1p_rs84_S131072_n4096 verify_all_rs84_S131072_n4096 get_into0_rs124_S87382_n4096 get_into2_rs124_S87382_n4096 heal_1d1p_rs124_S87382_n4096 verify_all_rs124_S87382_n4096"}
for key in $KEYS; do
  mkdir -p $OUT/$key
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d $OUT/$key/$c -o run --output-format csv \
      -- python3 $R/tools/pmc_driver.py $key $OUT/$key 3 > $OUT/$key/$c.log 2>&1 || { mkdir -p $OUT/$key; tail -5 $OUT/$key/$c.log; exit 1; }
    rm -f $OUT/$key/$c/run_agent_info.csv
  done
  echo "$key ok"
done
echo done
