#!/bin/bash
# Full GPU validation + measurements: all gpu tests, the lattice traces, the drop-in
# step (default and V-stream-only), the bench. Each step bounded; stop at the first failure.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 120 python tools/trace_lat.py build/libmfgp_stamps.so > gpurun_out/trace_b8.txt 2>&1 || { echo "trace failed"; tail gpurun_out/trace_b8.txt; exit 1; }
TRACE_B=1 timeout -k 10 120 python tools/trace_lat.py build/libmfgp_stamps.so > gpurun_out/trace_b1.txt 2>&1 || { echo "trace1 failed"; tail gpurun_out/trace_b1.txt; exit 1; }
grep -E "last WG end" gpurun_out/trace_b8.txt gpurun_out/trace_b1.txt
timeout -k 10 120 python tools/bench_dropin.py > gpurun_out/dropin.jsonl 2>&1 || { echo "dropin failed"; tail gpurun_out/dropin.jsonl; exit 1; }
MFGP_LATTICE=0 timeout -k 10 120 python tools/bench_dropin.py >> gpurun_out/dropin.jsonl 2>&1 || { echo "dropin0 failed"; tail gpurun_out/dropin.jsonl; exit 1; }
grep '^{' gpurun_out/dropin.jsonl
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench20.json 2> gpurun_out/bench20.err || { echo "bench failed"; tail -20 gpurun_out/bench20.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench20.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
