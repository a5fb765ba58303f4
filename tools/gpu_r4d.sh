#!/bin/bash
# Round-4 pass D: RS(12,4) network kernels with 6/6 halves and split
# finishing (every listed pattern, ragged walks), their kernel stats, the
# RS(12,4) line (encode with the layout-chosen workgroup size), the default
# line, and the kernel-timing hook against rocprof (tools/hook_check.py).
# Usage: bash tools/gpu_r4d.sh TAG
set -o pipefail
TAG=${1:-r4d}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode_nets.py tests/test_gpu_decode.py tests/test_gpu_async.py -x -q --timeout 170 --timeout-method thread -m gpu -k "rs12 or long or ragged or into or async or lost_disk" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
cd /tmp
for what in into2 heal; do
  EP_K=12 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/k12_$what -o run --output-format csv -- python3 $R/tools/engine_prof.py $what 10 > $OUT/k12_$what.txt 2>&1 || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/hook -o run --output-format csv -- python3 $R/tools/hook_check.py 8 > $OUT/hook.json 2> $OUT/hook.err || exit $?
cd $R
timeout -k 10 400 python -u bench.py --k 12 --m 4 --no-cpu-baseline --no-config-extras > $OUT/bench_12_4.json 2> $OUT/bench_12_4.err || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
cat $OUT/hook.json
echo done
