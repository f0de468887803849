#!/bin/bash
# g3: lattice parity, gemm3 timeline (stamps build), headline bench g3 vs g2
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lattice.py > gpurun_out/r04l_lat.log 2>&1 || { tail -30 gpurun_out/r04l_lat.log; exit 1; }
tail -1 gpurun_out/r04l_lat.log
MFGP_LAT_G3=1 timeout -k 10 200 python -u tools/trace_g3.py tools/diaglib/libmfgp_stamps.so || exit 1
MFGP_LAT_G3=1 timeout -k 10 300 python -u bench.py --sim-iterations 0 --no-cpu-baseline > gpurun_out/r04l_g3.json 2> gpurun_out/r04l_g3.err || exit $?
MFGP_LAT_G3=0 timeout -k 10 300 python -u bench.py --sim-iterations 0 --no-cpu-baseline > gpurun_out/r04l_g2.json 2> gpurun_out/r04l_g2.err || exit $?
python - <<'PY'
import json
for f in ("r04l_g3", "r04l_g2"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, round(d["value"]), round(1e3 * d["ms_per_step"], 2), round(d["roofline"]["frac"], 3))
PY
