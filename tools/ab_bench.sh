#!/bin/bash
# A/B of library variants on the headline bench (8 seeds) and the single-GP case,
# interleaved: tools/ab_bench.sh VARIANT... (default = the in-tree library)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
for rep in 1 2; do
for v in "$@"; do
  L=$R/build/libmfgp_$v.so
  [ "$v" = "default" ] && L=$R/mfgp_coverage_amd/libmfgp_hip.so
  for B in 8 1; do
    MFGP_LIB=$L timeout -k 10 120 python -u bench.py --diagnostic --seeds-per-gpu $B --no-full --no-cpu-baseline --steps 400 --warmup 40 \
      > gpurun_out/ab_${v}_$B.json 2> gpurun_out/ab_${v}_$B.err || { echo "$v failed"; tail -5 gpurun_out/ab_${v}_$B.err; exit 1; }
    python - "$v" $B gpurun_out/ab_${v}_$B.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[1]:>10} B={sys.argv[2]}: {d['value']:8.0f} upd/s {d['ms_per_step']*1e3:7.1f} us/step kernel {r['avg_launch_ms']*1e3:6.1f} us {r['achieved']:6.0f} GB/s")
PY
  done
done
done
