#!/bin/bash
# Per-pattern XOR-network GET/heal kernels: their parity tests, the decode /
# heal suites, then bench.py's engine extras with the networks on and off
# (RSG_DECODE_NET=0: run-time-table GF waves) and a rocprof kernel-stats run
# of the engine extras.  Usage: bash tools/gpu_nets.sh TAG [skip-tests]
. "$(dirname "$0")/measure_env.sh"  # RSG_* knobs: the measurement build (ABI 6)
set -o pipefail
TAG=${1:-r3_nets}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decode_nets.py \
    tests/test_gpu_decode.py tests/test_gpu_heal.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
for net in 1 0; do
  RSG_DECODE_NET=$net timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-config-extras --steps 5 \
    > $OUT/eng_net$net.json 2> $OUT/eng_net$net.err || exit $?
  python - $OUT/eng_net$net.json $net <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); g=d['extras']['engines']
print('net', sys.argv[2], {k:(v.get('kernel_ms'),v['frac']) for k,v in g.items() if isinstance(v,dict)}, flush=True)
PY
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o eng --output-format csv \
  -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-config-extras --steps 5 > $GRAFT_REPO_ROOT/$OUT/eng_prof.json 2> $GRAFT_REPO_ROOT/$OUT/prof.err
rc=$?
cd $GRAFT_REPO_ROOT
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/eng_kernel_stats.csv \;
exit $rc
