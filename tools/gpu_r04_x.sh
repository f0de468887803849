#!/bin/bash
# Z units reading the scan units' member lists (MFGP_LAT_ZCSR=1): lattice parity, then A/B at the headline and configs[4]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
MFGP_LAT_ZCSR=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_lattice.py tests/test_gpu_f32.py tests/test_gpu_lattice_reference.py tests/test_gpu_headline.py > gpurun_out/r04x_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r04x_tests.log | head; tail -25 gpurun_out/r04x_tests.log; exit 1; }
tail -1 gpurun_out/r04x_tests.log
for rep in 1 2; do
  for z in 0 1; do
    MFGP_LAT_ZCSR=$z timeout -k 10 300 python bench.py --no-full --no-cpu-baseline --sim-iterations 0 > gpurun_out/r04x_h${z}_$rep.json 2>/dev/null || exit 1
    MFGP_LAT_ZCSR=$z timeout -k 10 300 python bench.py --workload configs4 --no-full --no-cpu-baseline --sim-iterations 0 > gpurun_out/r04x_c${z}_$rep.json 2>/dev/null || exit 1
    python -c "
import json
for f in ('h${z}_$rep', 'c${z}_$rep'):
    d=json.load(open(f'gpurun_out/r04x_{f}.json')); print(f, round(d['value']), round(1e3*d['ms_per_step'],2), round(1e3*d['roofline']['avg_launch_ms'],2))"
  done
done
