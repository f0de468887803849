#!/bin/bash
# round-4: the whole GPU suite + smoke
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu tests/ > gpurun_out/r04_gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r04_gpu_tests.log
grep -E "FAILED|ERROR" gpurun_out/r04_gpu_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
