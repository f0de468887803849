#!/bin/bash
# round-4: kernel trace of the headline step (gaps between the two launches and steps)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_r04f
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r04f/trace -o bench -- \
  python3 $R/bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-full --sim-iterations 0 > $R/gpurun_out/prof_r04f/trace.log 2>&1 || exit $?
cd $R
f=$(ls gpurun_out/prof_r04f/trace/*kernel_trace.csv | head -1)
python tools/step_gaps.py $f
head -8 gpurun_out/prof_r04f/trace/*kernel_stats.csv
