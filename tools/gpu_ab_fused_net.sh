#!/bin/bash
# The fused encode + HH256S on the network kernels (B: RS(10,4) on the
# four-wave netq kernel, RS(6,4) / RS(4,4) on the 8-stripe one) against the
# packed table kernel (A): the GPU suite on B, then bench.py's line for each
# geometry with --digests, A B A B A B (tools/ab_libs.sh), and RS(8,4) with
# the network kernel forced against its LDS-DMA kernel on B.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab_fused_net
mkdir -p $OUT
RSG_LIB_PATH=$R/rustfs_amd/ab/B.so timeout -k 10 600 python -u -m pytest tests -x -q --timeout 60 --timeout-method thread -m gpu > $OUT/pytest_gpu_B.log 2>&1 || { tail -30 $OUT/pytest_gpu_B.log; exit 1; }
tail -1 $OUT/pytest_gpu_B.log
for k in 10 6 4; do
  bash tools/ab_libs.sh ab_fused_net/k$k "--k $k --m 4 --digests --no-extras --no-cpu-baseline --no-rs12" || exit 1
done
echo done
