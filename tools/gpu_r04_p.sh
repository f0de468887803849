#!/bin/bash
# coverage drivers after the indexed sampling: GPU coverage tests, then the bench's simulation leg
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_coverage.py > gpurun_out/r04p2_cov.log 2>&1 || { tail -30 gpurun_out/r04p2_cov.log; exit 1; }
tail -1 gpurun_out/r04p2_cov.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-full > gpurun_out/r04p2_bench.json 2> gpurun_out/r04p2_bench.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/r04p2_bench.json')); s=d['simulation']; print(round(d['value']), s['value'], s['ms_per_iteration'], s['breakdown_ms_per_iteration'], s['dropin_one_seed'])"
# w units over the batch (MFGP_LAT_WU; the host's rule gives 512 at the headline)
for wu in 512 768 1024 512 768; do
  MFGP_LAT_WU=$wu timeout -k 10 300 python -u bench.py --sim-iterations 0 --no-cpu-baseline --no-full > gpurun_out/r04p2_wu$wu.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/r04p2_wu$wu.json')); print('wu $wu', round(d['value']), round(1e3*d['ms_per_step'],2))"
done
