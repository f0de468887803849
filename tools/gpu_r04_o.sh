#!/bin/bash
# drop-in step: blocking stream sync (default) vs hipStreamQuery polling (MFGP_SYNC_QUERY=1), alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04o
for rnd in 1 2; do
  for q in 0 1; do
    MFGP_SYNC_QUERY=$q timeout -k 10 120 python -u tools/bench_dropin.py > gpurun_out/r04o/bd_q${q}_$rnd.json 2>/dev/null || exit 1
    MFGP_SYNC_QUERY=$q timeout -k 10 120 python -u tools/dropin_r04.py > gpurun_out/r04o/dr_q${q}_$rnd.json 2>/dev/null || exit 1
    echo "q=$q r=$rnd $(cat gpurun_out/r04o/bd_q${q}_$rnd.json | cut -c1-150)"
    echo "      $(cat gpurun_out/r04o/dr_q${q}_$rnd.json | cut -c40-260)"
  done
done
