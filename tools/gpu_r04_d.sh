#!/bin/bash
# round-4: short-window timing probe; drop-in step with / without the status poll
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/window_probe.py > gpurun_out/r04d_window.json 2>/dev/null || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r04d_window.json"))
for k, v in d.items():
    print(k, [round(r["us_per_step"], 1) for r in v], [(round(r.get("first_step_us", 0), 1), round(r.get("last_step_us", 0), 1), round(r.get("gpu_span_us", 0), 1), round(r.get("wall_us", 0), 1)) for r in v if "first_step_us" in r])
PY
for sp in 0 2000; do
  MFGP_SPIN_US=$sp timeout -k 10 120 python -u tools/dropin_r04.py > gpurun_out/r04d_dropin_spin$sp.json 2>/dev/null || exit $?
  echo spin=$sp; cat gpurun_out/r04d_dropin_spin$sp.json
done
