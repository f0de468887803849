#!/bin/bash
# Single-GP paths (the drop-in simulator's case: one GP per process) across library variants:
# bench.py with one seed (k = 8 appends), and the Choi planner loop (k = 1 appends).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for v in "$@"; do
  L=$R/build/libmfgp_$v.so
  [ "$v" = "default" ] && L=$R/mfgp_coverage_amd/libmfgp_hip.so
  MFGP_LIB=$L timeout -k 10 120 python -u bench.py --diagnostic --seeds-per-gpu 1 --no-full --no-cpu-baseline --steps 300 --warmup 30 \
    > gpurun_out/single_$v.json 2> gpurun_out/single_$v.err || { echo "$v failed"; tail -5 gpurun_out/single_$v.err; exit 1; }
  python - "$v" gpurun_out/single_$v.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[1]:>10} B=1: {d['value']:8.0f} upd/s {d['ms_per_step']*1e3:7.1f} us/step kernel {r['avg_launch_ms']*1e3:6.1f} us {r['achieved']:6.0f} GB/s")
PY
  MFGP_LIB=$L timeout -k 10 120 python -u tools/bench_planner.py 2>/dev/null | tail -1 || { echo "$v planner failed"; exit 1; }
done
