#!/bin/bash
# round-4 evidence: headline bench (driver form and default), configs[4] bench,
# rocprofv3 kernel trace + PMC passes of the headline
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/r04p_bench_default.json 2> gpurun_out/r04p_bench_default.err || exit $?
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r04p_bench20.json 2> gpurun_out/r04p_bench20.err || exit $?
timeout -k 10 600 python -u bench.py --workload configs4 > gpurun_out/r04p_configs4.json 2> gpurun_out/r04p_configs4.err || exit $?
python - <<'PY'
import json
for f in ("r04p_bench_default", "r04p_bench20", "r04p_configs4"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, round(d["value"]), round(1e3 * d["ms_per_step"], 2), round(d["roofline"]["frac"], 3),
          d.get("full_recompute", {}).get("value"), d.get("cpu_baseline", {}).get("value"))
PY
bash tools/profile_round.sh r04 > gpurun_out/r04p_prof.log 2>&1 || exit $?
python tools/summarize_profile.py gpurun_out/prof_r04 r04 > gpurun_out/r04p_summary.txt 2>&1
tail -40 gpurun_out/r04p_summary.txt
# the two-launch step's per-workgroup timeline (stamps build; k_lat_gemm2 by XCD)
timeout -k 10 200 python -u tools/trace_lat.py tools/diaglib/libmfgp_stamps.so > gpurun_out/r04p_trace_lat.txt 2>&1 || true
