#!/bin/bash
# One lattice iteration on the box: the lattice tests, the B = 8 / B = 1 traces
# (build/libmfgp_stamps.so) and a short bench. Each step bounded; stop at the first failure.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_lattice.py tests/test_gpu_lattice_reference.py ${LAT_TESTS:-} -x -q --timeout 120 --timeout-method thread > gpurun_out/lat_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/lat_tests.log; exit 1; }
tail -2 gpurun_out/lat_tests.log
timeout -k 10 120 python tools/trace_lat.py build/libmfgp_stamps.so > gpurun_out/trace_b8.txt 2>&1 || { echo "trace failed"; tail gpurun_out/trace_b8.txt; exit 1; }
TRACE_B=1 timeout -k 10 120 python tools/trace_lat.py build/libmfgp_stamps.so > gpurun_out/trace_b1.txt 2>&1 || { echo "trace1 failed"; tail gpurun_out/trace_b1.txt; exit 1; }
head -30 gpurun_out/trace_b8.txt; head -30 gpurun_out/trace_b1.txt
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 > gpurun_out/bench_iter.json 2> gpurun_out/bench_iter.err || { echo "bench failed"; tail -20 gpurun_out/bench_iter.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_iter.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
