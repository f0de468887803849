#!/bin/bash
# A/B of library variants (tools/stamps_lib/libmfgp_<v>.so) at configs[4] (bench.py
# --workload configs4, incremental leg), alternating, twice.
# usage (GPU box): bash tools/ab_libs_c4.sh default v1 v2 ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
for rep in 1 2; do
for v in "$@"; do
  L=$R/tools/stamps_lib/libmfgp_$v.so
  [ "$v" = "default" ] && L=$R/mfgp_coverage_amd/libmfgp_hip.so
  MFGP_LIB=$L timeout -k 10 200 python -u bench.py --diagnostic --workload configs4 --no-full --no-cpu-baseline --steps 40 --warmup 5 --sim-iterations 0 > gpurun_out/abc4_$v.json 2> gpurun_out/abc4_$v.err || { echo "$v failed rc=$?"; tail -5 gpurun_out/abc4_$v.err; exit 1; }
  python3 - "$v" gpurun_out/abc4_$v.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"c4 {sys.argv[1]:>10}: {d['value']:9.0f} upd/s  {d['ms_per_step']*1e3:7.1f} us/step  kernel {r['avg_launch_ms']*1e3:7.1f} us")
PY
done
done
