#!/bin/bash
# round-4 check: the new coverage / headline tests, then a short bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_coverage.py tests/test_gpu_headline.py "tests/test_gpu_incremental.py::test_headline_batch_default_step_vs_full" \
  tests/test_sharded.py tests/test_boundary.py > gpurun_out/r04a_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r04a_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r04a_bench20.json 2> gpurun_out/r04a_bench20.err
rc=$?
tail -c 3000 gpurun_out/r04a_bench20.json
exit $rc
