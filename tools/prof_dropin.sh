#!/bin/bash
# Kernel stats of the drop-in step, lattice (default) and V stream (MFGP_LATTICE=0)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dropin_lat -o run -- python3 tools/bench_dropin.py > gpurun_out/prof_dropin_lat.log 2>&1 || exit 1
MFGP_LATTICE=0 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dropin_vs -o run -- python3 tools/bench_dropin.py > gpurun_out/prof_dropin_vs.log 2>&1 || exit 1
for d in lat vs; do f=$(find gpurun_out/prof_dropin_$d -name "*kernel_stats.csv" | head -1); echo "== $d"; head -8 "$f" | cut -c1-200; done
