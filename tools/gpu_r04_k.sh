#!/bin/bash
# g3: parity of the gemm3 tests, then the per-workgroup gemm3 timeline (stamps build)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lattice.py -k "gemm3 or gemm2" > gpurun_out/r04k_lat.log 2>&1 || { tail -30 gpurun_out/r04k_lat.log; exit 1; }
tail -1 gpurun_out/r04k_lat.log
timeout -k 10 200 python -u tools/trace_g3.py tools/diaglib/libmfgp_stamps.so
