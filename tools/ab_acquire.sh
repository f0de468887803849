#!/bin/bash
# A/B of the hand-off acquire: bench.py and the drop-in step with
# build/libmfgp_acq.so (an agent-scope acquire after every flag wait:
#   python -c "import __graft_entry__ as g; g.build(extra=['-DMFGP_ACQUIRE'], out='build/libmfgp_acq.so')")
# and the default library (relaxed polls), twice each, alternating. Output under
# gpurun_out/ab_acq/.
set -e
mkdir -p gpurun_out/ab_acq
for rep in 1 2; do
  for v in acq noacq; do
    if [ $v = acq ]; then export MFGP_LIB=build/libmfgp_acq.so; D=--diagnostic; else unset MFGP_LIB; D=; fi
    timeout -k 10 240 python bench.py --gpus 1 --steps ${STEPS:-200} --warmup 10 $D > gpurun_out/ab_acq/bench_${v}_$rep.json 2> gpurun_out/ab_acq/bench_${v}_$rep.err
    timeout -k 10 120 python tools/bench_dropin.py > gpurun_out/ab_acq/dropin_${v}_$rep.txt 2>&1
    echo "$v $rep done"
  done
done
unset MFGP_LIB
