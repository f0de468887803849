#!/bin/bash
# GPU box: HIP API + kernel trace of the drop-in step (tools/bench_dropin.py), for
# the host-side cost of each runtime call. No counters in this pass.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/trace_dropin
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $OUT -o dropin -- \
  python3 $R/tools/bench_dropin.py > $OUT/run.log 2>&1
tail -2 $OUT/run.log
