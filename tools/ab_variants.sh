#!/bin/bash
# A/B of library variants (tools/diaglib/libmfgp_<v>.so, built in the build
# container) against the default library: the headline bench, alternating, twice.
# usage: bash tools/ab_variants.sh v1 v2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab_var
for rep in 1 2; do
  for v in default "$@"; do
    if [ $v = default ]; then unset MFGP_LIB; D=; else export MFGP_LIB=tools/diaglib/libmfgp_$v.so; D=--diagnostic; fi
    timeout -k 10 240 python bench.py --steps 300 --warmup 10 --no-full --no-cpu-baseline --sim-iterations 0 $D \
      > gpurun_out/ab_var/bench_${v}_$rep.json 2> gpurun_out/ab_var/bench_${v}_$rep.err || exit $?
    python -c "import json;d=json.load(open('gpurun_out/ab_var/bench_${v}_$rep.json'));print('$v $rep', round(d['value']), round(1e3*d['ms_per_step'],2), round(1e3*d['roofline']['avg_launch_ms'],2))"
  done
done
unset MFGP_LIB
