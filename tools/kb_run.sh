#!/bin/bash
# Run one tools/kbench binary on the GPU box with its own time limit.
# Usage: bash tools/kb_run.sh TAG BINARY [args...]
set -o pipefail
TAG=$1; BIN=$2; shift 2
mkdir -p gpurun_out/$TAG
timeout -k 10 300 tools/kbench/$BIN "$@" > gpurun_out/$TAG/$BIN.txt 2>&1
rc=$?
cat gpurun_out/$TAG/$BIN.txt
exit $rc
