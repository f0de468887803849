#!/bin/bash
# one GP: the lattice step forced vs the V stream, back to back and with 40 us host pauses (kernel durations)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r04q
export TMPDIR=/tmp
cd /tmp
for mode in lat vs; do
  for p in 0 40; do
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04q/${mode}_p$p -o b -- \
      python3 $R/tools/probe_b1.py $p $mode > $R/gpurun_out/r04q/${mode}_p$p.log 2>&1 || exit 1
    echo "== $mode pause $p: $(grep pause_us $R/gpurun_out/r04q/${mode}_p$p.log | cut -c1-50)"
    grep "inc_stream1\|inc_lat\|gemm2" $R/gpurun_out/r04q/${mode}_p$p/b_kernel_stats.csv | cut -d, -f1-7
  done
done
