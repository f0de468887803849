#!/bin/bash
# g3 (the second launch builds its own Z rows): lattice parity, headline chain,
# coverage; then the headline bench with g3 (default) and g2 (MFGP_LAT_G3=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 500 $PYT tests/test_gpu_lattice.py > gpurun_out/r04h_lattice.log 2>&1 || { tail -30 gpurun_out/r04h_lattice.log; exit 1; }
tail -3 gpurun_out/r04h_lattice.log
timeout -k 10 400 $PYT tests/test_gpu_incremental.py -k headline > gpurun_out/r04h_inc.log 2>&1 || { tail -30 gpurun_out/r04h_inc.log; exit 1; }
tail -2 gpurun_out/r04h_inc.log
timeout -k 10 600 python -u bench.py --sim-iterations 0 > gpurun_out/r04h_g3.json 2> gpurun_out/r04h_g3.err || exit $?
MFGP_LAT_G3=0 timeout -k 10 600 python -u bench.py --sim-iterations 0 > gpurun_out/r04h_g2.json 2> gpurun_out/r04h_g2.err || exit $?
python - <<'PY'
import json
for f in ("r04h_g3", "r04h_g2"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, round(d["value"]), round(1e3 * d["ms_per_step"], 2), round(d["roofline"]["frac"], 3), d["roofline"].get("achieved"))
PY
timeout -k 10 1000 $PYT --timeout 1100 tests/test_gpu_headline.py tests/test_gpu_coverage.py > gpurun_out/r04h_head.log 2>&1 || { tail -30 gpurun_out/r04h_head.log; exit 1; }
tail -3 gpurun_out/r04h_head.log
