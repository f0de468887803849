#!/bin/bash
# tools/bench_stream_modes.py across library variants (build/libmfgp_*.so; "default" = the product build)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for v in "$@"; do
  L=$R/build/libmfgp_$v.so
  [ "$v" = "default" ] && L=$R/mfgp_coverage_amd/libmfgp_hip.so
  echo "== $v"
  MFGP_LIB=$L timeout -k 10 120 python -u tools/bench_stream_modes.py 2>/dev/null || { echo "$v failed"; exit 1; }
done
