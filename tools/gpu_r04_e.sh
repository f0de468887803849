#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/dropin_r04.py > gpurun_out/r04e_dropin.json 2>/dev/null || exit $?
cat gpurun_out/r04e_dropin.json
timeout -k 10 120 python -u tools/bench_dropin.py > gpurun_out/r04e_bench_dropin.json 2>/dev/null || exit $?
cat gpurun_out/r04e_bench_dropin.json
timeout -k 10 300 python -u bench.py --no-full --no-cpu-baseline --sim-iterations 0 > gpurun_out/r04e_bench200.json 2>/dev/null || exit $?
python -c "import json;d=json.load(open('gpurun_out/r04e_bench200.json'));print('bench200', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'])"
bash tools/ab_narrow.sh
