#!/bin/bash
# A/B the bench's incremental step across library variants (build/libmfgp_*.so).
# usage (GPU box): bash tools/ab_libs.sh name1 name2 ...   (each run bounded)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
for rep in 1 2; do
for v in "$@"; do
  L=$R/tools/stamps_lib/libmfgp_$v.so; [ -f "$L" ] || L=$R/build/libmfgp_$v.so
  [ "$v" = "default" ] && L=$R/mfgp_coverage_amd/libmfgp_hip.so
  MFGP_LIB=$L timeout -k 10 120 python -u bench.py --diagnostic --no-full --no-cpu-baseline --steps 300 --warmup 30 > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo "$v failed rc=$?"; tail -5 gpurun_out/ab_$v.err; exit 1; }
  python - "$v" gpurun_out/ab_$v.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[1]:>10}: {d['value']:9.0f} upd/s  {d['ms_per_step']*1e3:7.1f} us/step  kernel {r['avg_launch_ms']*1e3:7.1f} us  {r['achieved']:7.0f} GB/s  frac {r['frac']:.3f}")
PY
done
done
