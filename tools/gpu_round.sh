#!/bin/bash
# Round pass: GPU tests, smoke, default bench (with CPU baseline), PCIe rates,
# 2-rank rehearsal on one GPU, rocprof kernel stats.  Each GPU step has its own
# time limit; steps chained with && so a failure ends the call.
set -o pipefail
TAG=${1:-round}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $OUT/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
 && timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err \
 && timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras --digests > $OUT/bench_fused.json 2>> $OUT/bench.err \
 && timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras --k 16 --m 4 > $OUT/bench_16_4.json 2>> $OUT/bench.err \
 && timeout -k 10 300 python tools/engine_bench.py > $OUT/engine.json 2> $OUT/engine.err \
 && timeout -k 10 300 python tools/pcie_bench.py > $OUT/pcie.json 2> $OUT/pcie.err \
 && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --batch 1024 --no-extras > $OUT/bench_2rank_rehearsal.json 2> $OUT/bench2.err \
 && cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/bench_prof.json 2> $GRAFT_REPO_ROOT/$OUT/prof.err \
 && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof_fused -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras --digests > $GRAFT_REPO_ROOT/$OUT/bench_prof_fused.json 2>> $GRAFT_REPO_ROOT/$OUT/prof.err
