#!/bin/bash
# compact-row loads of the w units without the unused lanes' lines: lattice tests, headline and configs[4]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lattice.py tests/test_gpu_f32.py > gpurun_out/r04w_tests.log 2>&1 || { tail -20 gpurun_out/r04w_tests.log; exit 1; }
tail -1 gpurun_out/r04w_tests.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --no-full --no-cpu-baseline --sim-iterations 0 > gpurun_out/r04w_h$rep.json 2>/dev/null || exit 1
  timeout -k 10 300 python bench.py --workload configs4 --no-full --no-cpu-baseline --sim-iterations 0 > gpurun_out/r04w_c$rep.json 2>/dev/null || exit 1
  python -c "
import json
for f in ('h$rep', 'c$rep'):
    d=json.load(open(f'gpurun_out/r04w_{f}.json')); print(f, round(d['value']), round(1e3*d['ms_per_step'],2), round(1e3*d['roofline']['avg_launch_ms'],2))"
done
