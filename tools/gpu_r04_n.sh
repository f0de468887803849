#!/bin/bash
# one GP's V stream (k_inc_stream1): back to back vs with 40 us host pauses, row splits 4 (default) / 2 / 1
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r04n
export TMPDIR=/tmp
cd /tmp
for rs in 0 2 1; do
  for p in 0 40; do
    MFGP_RSPLIT=$rs timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04n/r${rs}_p$p -o b -- \
      python3 $R/tools/probe_b1.py $p > $R/gpurun_out/r04n/r${rs}_p$p.log 2>&1 || exit 1
    echo "== rsplit $rs pause $p: $(grep pause_us $R/gpurun_out/r04n/r${rs}_p$p.log | cut -c1-60)"
    grep inc_stream1 $R/gpurun_out/r04n/r${rs}_p$p/b_kernel_stats.csv | cut -d, -f1-7
  done
done
