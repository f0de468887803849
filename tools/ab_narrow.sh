#!/bin/bash
# A/B of the narrow hand-off acquire: the
# headline bench and the drop-in step with tools/variants/libmfgp_narrow.so
# (-DMFGP_ACQUIRE_NARROW: one agent-scope acquire per wait, by the polling wave)
# and the default library, twice each, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab_narrow
for rep in 1 2; do
  for v in narrow default; do
    if [ $v = narrow ]; then export MFGP_LIB=tools/variants/libmfgp_narrow.so; D=--diagnostic; else unset MFGP_LIB; D=; fi
    timeout -k 10 240 python bench.py --steps 200 --warmup 10 --no-full --no-cpu-baseline --sim-iterations 0 $D \
      > gpurun_out/ab_narrow/bench_${v}_$rep.json 2> gpurun_out/ab_narrow/bench_${v}_$rep.err || exit $?
    timeout -k 10 120 python tools/bench_dropin.py > gpurun_out/ab_narrow/dropin_${v}_$rep.json 2>/dev/null || exit $?
    python -c "import json;d=json.load(open('gpurun_out/ab_narrow/bench_${v}_$rep.json'));e=json.load(open('gpurun_out/ab_narrow/dropin_${v}_$rep.json'));print('$v $rep', round(d['value']), round(1e3*d['ms_per_step'],1), round(1e3*d['roofline']['avg_launch_ms'],1), e['us_median'])"
  done
done
unset MFGP_LIB
