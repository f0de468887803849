#!/bin/bash
# A/B of lattice-step environment switches on one box: the lattice tests once, then
# a 200-step bench per setting, alternating twice. usage: bash tools/ab_lat_env.sh "A=1" "A=2 B=3" ...
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_lattice.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lat_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/lat_tests.log; exit 1; }
tail -1 gpurun_out/lat_tests.log
for rep in 1 2; do
  for cfg in "$@"; do
    env $cfg timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --no-full --no-cpu-baseline --diagnostic > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "bench failed: $cfg"; tail -20 gpurun_out/ab.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print(sys.argv[1], round(d['value']), round(1e3*d['ms_per_step'],2), round(1e3*d['roofline']['avg_launch_ms'],2))" "$cfg"
  done
done
