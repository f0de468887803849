#!/bin/bash
# configs[4] with fp32 F: w-unit count and the two-launch GEMM
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04t
for v in "MFGP_LAT_WU=1024" "MFGP_LAT_WU=2048" "MFGP_LAT_WU=4096" "MFGP_LAT_GEMM2=1" "X=0"; do
  env $v timeout -k 10 300 python -u bench.py --workload configs4 --no-cpu-baseline --no-full --sim-iterations 0 > gpurun_out/r04t/c4_${v}.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/r04t/c4_${v}.json')); print('$v', round(d['value']), round(1e3*d['ms_per_step'],1), round(1e3*d['roofline']['avg_launch_ms'],1))"
done
