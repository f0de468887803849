#!/bin/bash
# configs[4] evidence with fp32 F: bench + rocprofv3 kernel trace / PMC passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --workload configs4 > gpurun_out/r04u_configs4.json 2> gpurun_out/r04u_configs4.err || exit 1
bash tools/profile_round.sh r04_configs4 --workload configs4 > gpurun_out/r04u_prof.log 2>&1 || exit 1
echo done
