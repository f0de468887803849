#!/bin/bash
# kernel durations of the headline step, g3 vs g2 (rocprofv3 kernel trace)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r04i
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04i/g3 -o b -- \
  python3 $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-full --sim-iterations 0 > $R/gpurun_out/r04i/g3.log 2>&1 || exit $?
MFGP_LAT_G3=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04i/g2 -o b -- \
  python3 $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-full --sim-iterations 0 > $R/gpurun_out/r04i/g2.log 2>&1 || exit $?
for v in g3 g2; do f=$(ls $R/gpurun_out/r04i/$v/*/*kernel_stats.csv 2>/dev/null || ls $R/gpurun_out/r04i/$v/*kernel_stats.csv); echo "== $v"; cut -d, -f1-8 $f | head -8; done
