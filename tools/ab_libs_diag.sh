#!/bin/bash
# A/B of library builds on the default bench (incremental leg, --diagnostic so that
# MFGP_LIB is honoured; every run, the default build included, goes through it):
#   bash tools/ab_libs_diag.sh "lib1.so lib2.so ..." [rounds]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/ablib
LIBS=$1; ROUNDS=${2:-2}
for r in $(seq 1 $ROUNDS); do
  for l in $LIBS; do
    n=$(basename $l .so)
    MFGP_LIB=$R/$l timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 --no-full --no-cpu-baseline --diagnostic \
      > gpurun_out/ablib/${n}_$r.json 2> gpurun_out/ablib/${n}_$r.err || { echo "run $l failed"; tail -20 gpurun_out/ablib/${n}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), round(d['ms_per_step']*1e3,1), round(d['roofline']['avg_launch_ms']*1e3,1))" \
      gpurun_out/ablib/${n}_$r.json "$n"
  done
done
