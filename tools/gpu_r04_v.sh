#!/bin/bash
# configs[4]: w-unit steps in flight with fp32 F (default 10; df6 = the fp64 depth; df14), alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04v
for rep in 1 2; do
  for v in default df6 df14; do
    if [ $v = default ]; then unset MFGP_LIB; D=; else export MFGP_LIB=tools/diaglib/libmfgp_$v.so; D=--diagnostic; fi
    timeout -k 10 300 python bench.py --workload configs4 --no-full --no-cpu-baseline --sim-iterations 0 $D > gpurun_out/r04v/c4_${v}_$rep.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/r04v/c4_${v}_$rep.json'));print('$v $rep', round(d['value']), round(1e3*d['ms_per_step'],1), round(1e3*d['roofline']['avg_launch_ms'],1))"
  done
done
unset MFGP_LIB
