#!/bin/bash
# g3 parity (lattice tests) then kernel durations g3 vs g2 (rocprofv3 kernel trace)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r04j
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_lattice.py -k "gemm3 or gemm2 or headline" > gpurun_out/r04j/lat.log 2>&1 || { tail -30 gpurun_out/r04j/lat.log; exit 1; }
tail -2 gpurun_out/r04j/lat.log
export TMPDIR=/tmp
cd /tmp
for v in g3 g2; do
  if [ $v = g2 ]; then export MFGP_LAT_G3=0; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04j/$v -o b -- \
    python3 $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-full --sim-iterations 0 > $R/gpurun_out/r04j/$v.log 2>&1 || exit $?
  echo "== $v"; cut -d, -f1-8 $R/gpurun_out/r04j/$v/b_kernel_stats.csv | sed -n 2,3p
  grep '"metric"' $R/gpurun_out/r04j/$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), round(1e3*d['ms_per_step'],2))"
done
