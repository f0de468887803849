#!/bin/bash
# Quick A/B: the lattice tests, a 200-step bench, and the kernel trace gaps of the lattice step.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_lattice.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lat_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/lat_tests.log; exit 1; }
tail -1 gpurun_out/lat_tests.log
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --no-full --no-cpu-baseline > gpurun_out/qb.json 2> gpurun_out/qb.err || { echo "bench failed"; tail -20 gpurun_out/qb.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/qb.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['host_enqueue_ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/qbt -o t -- python3 bench.py --steps 100 --warmup 10 --no-full --no-cpu-baseline > gpurun_out/qbt.log 2>&1 || { echo "trace failed"; exit 1; }
python tools/step_gaps.py gpurun_out/qbt/t_kernel_trace.csv
