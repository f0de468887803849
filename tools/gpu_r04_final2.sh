#!/bin/bash
# round-4 close: whole GPU suite + smoke + headline bench (default and the driver's 20 steps)
# after the look-ahead factor change (ctx_create, enqueue_factor); kernels unchanged
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu tests/ > gpurun_out/r04_close_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r04_close_gpu_tests.log
grep -E "FAILED|ERROR" gpurun_out/r04_close_gpu_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r04_close_bench20.json 2> gpurun_out/r04_close_bench20.err || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r04_close_bench.json 2> gpurun_out/r04_close_bench.err || exit 1
python3 -c "
import json
for f in ('r04_close_bench20', 'r04_close_bench'):
    d = json.load(open(f'gpurun_out/{f}.json')); print(f, round(d['value']), round(1e3*d['ms_per_step'], 2), round(d['roofline']['frac'], 3), d.get('full_recompute', {}).get('breakdown_ms_per_step'))"
