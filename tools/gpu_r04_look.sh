#!/bin/bash
# round 4: look-ahead factor -- bit-equality tests, then factor ms per schedule
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_factor.py > gpurun_out/look_tests.log 2>&1
: > gpurun_out/look_factor.jsonl
for cfg in "0 64" "1 0" "1 32" "1 64" "1 96" "1 128" "0 64" "1 64"; do
  set -- $cfg
  echo "look=$1 crit=$2" >> gpurun_out/look_factor.jsonl
  MFGP_FACTOR_LOOKAHEAD=$1 MFGP_FACTOR_CRIT_CUS=$2 timeout -k 10 180 python tools/bench_factor.py --steps 10 >> gpurun_out/look_factor.jsonl
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MFGP_FACTOR_LOOKAHEAD=1 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/look_trace -o look -- python tools/bench_factor.py --steps 3 > gpurun_out/look_trace.log 2>&1
cat gpurun_out/look_factor.jsonl
