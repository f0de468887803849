#!/bin/bash
# fp32 F for MFGP_F32 models: fp32 / lattice / long-horizon tests, then configs[4]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_f32.py tests/test_gpu_lattice.py tests/test_gpu_long_horizon.py > gpurun_out/r04s_tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/r04s_tests.log | head -20; tail -30 gpurun_out/r04s_tests.log; exit 1; }
tail -1 gpurun_out/r04s_tests.log
timeout -k 10 600 python -u bench.py --workload configs4 > gpurun_out/r04s_configs4.json 2> gpurun_out/r04s_configs4.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/r04s_configs4.json')); print(round(d['value']), round(1e3*d['ms_per_step'],1), d['roofline'])"
