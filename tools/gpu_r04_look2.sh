#!/bin/bash
# round 4: look-ahead factor -- kernel trace of the factor stages (timeline overlap)
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MFGP_FACTOR_LOOKAHEAD=1 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/look_trace -o look -- python tools/bench_factor.py --steps 3 > gpurun_out/look_trace.log 2>&1
