#!/bin/bash
# rocprofv3 evidence of the full-path factor (tools/bench_factor.py: 8 GPs, N = 2048):
# kernel trace + stats, then the MFMA busy counters in a pass of their own.
# usage (GPU box): bash tools/profile_factor.sh
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_r05_factor
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o f -- python3 $R/tools/bench_factor.py > $OUT/trace.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/mfma -o f -- python3 $R/tools/bench_factor.py --steps 3 > $OUT/mfma.log 2>&1
echo done
