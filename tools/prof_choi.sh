#!/bin/bash
# Kernel trace + stats of the batched Choi selection (tools/bench_planner.py --batch 8):
# which kernels one batched iteration launches and how long each runs.
# usage (on the GPU box): bash tools/prof_choi.sh TAG [bench_planner args]
set -e
TAG=${1:-choi}
shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o choi -- \
  python3 $R/tools/bench_planner.py --batch 8 "$@" > $OUT/trace.log 2>&1
echo done
