#!/bin/bash
# staged CSR Z units: equality tests, configs[4] tests, then configs[4] twice
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_lattice.py tests/test_gpu_f32.py > gpurun_out/r04z_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r04z_tests.log | head; tail -25 gpurun_out/r04z_tests.log; exit 1; }
tail -1 gpurun_out/r04z_tests.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --workload configs4 --no-full --no-cpu-baseline --sim-iterations 0 > gpurun_out/r04z_c$rep.json 2>/dev/null || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/r04z_c$rep.json')); print('c$rep', round(d['value']), round(1e3*d['ms_per_step'],1), round(1e3*d['roofline']['avg_launch_ms'],1))"
done
