#!/bin/bash
# A/B of library variants on the drop-in step (tools/bench_dropin.py), alternating.
# usage (GPU box): bash tools/ab_dropin.sh default v1 ...   (tools/stamps_lib/libmfgp_<v>.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
for rep in 1 2 3; do
for v in "$@"; do
  L=$R/tools/stamps_lib/libmfgp_$v.so
  [ "$v" = "default" ] && L=$R/mfgp_coverage_amd/libmfgp_hip.so
  MFGP_LIB=$L timeout -k 10 120 python -u tools/bench_dropin.py > gpurun_out/abd_$v.json 2> gpurun_out/abd_$v.err || { echo "$v failed"; tail -5 gpurun_out/abd_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); u=d['us_median']; print(sys.argv[2], u, round(sum(u.values()),1))" gpurun_out/abd_$v.json $v
done
done
