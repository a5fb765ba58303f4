#!/bin/bash
# Round-4 final pass: the whole GPU suite, smoke, the default bench line
# (BASELINE metric + config 3/4/5 + engines + CPU baseline), the RS(12,4)
# lines (encode; encode + fused HH256S), and a rocprof kernel-stats run of
# the default command whose per-kernel averages must agree with the line's
# kernel_ms.  Each GPU step has its own time limit; && ends the call at the
# first failure.  Usage: bash tools/gpu_r4final.sh TAG
set -o pipefail
TAG=${1:-r4final}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "host: $(hostname) nproc: $(nproc)" > $OUT/env.txt
timeout -k 10 700 python -u -m pytest tests -x -q --timeout 170 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 \
 && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 400 python -u bench.py --k 12 --m 4 --no-cpu-baseline --no-config-extras > $OUT/bench_12_4.json 2> $OUT/bench_12_4.err || exit 1
timeout -k 10 400 python -u bench.py --k 12 --m 4 --digests --no-extras --no-cpu-baseline > $OUT/bench_12_4_digests.json 2> $OUT/bench_12_4_digests.err || exit 1
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
for what in into2 heal into0; do
  EP_K=12 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/k12_$what -o run --output-format csv -- python3 $R/tools/engine_prof.py $what 10 > $OUT/k12_$what.txt 2>&1 || exit 1
done
cat $OUT/bench.json
echo done
