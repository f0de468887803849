#!/bin/bash
# A/B of an environment switch on the default bench (incremental leg only):
#   bash tools/ab_env.sh VAR "valA valB" [rounds] [extra bench args]
# Alternates the values `rounds` times (box drift shows up as spread, not bias);
# prints GP-updates/s, us per step and us per launch of the dominant kernel per run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/ab
VAR=$1; VALS=$2; ROUNDS=${3:-2}; shift 3 || shift $#
for r in $(seq 1 $ROUNDS); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 --no-full --no-cpu-baseline "$@" \
      > gpurun_out/ab/${VAR}_${v}_$r.json 2> gpurun_out/ab/${VAR}_${v}_$r.err || { echo "run $VAR=$v failed"; tail -20 gpurun_out/ab/${VAR}_${v}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), round(d['ms_per_step']*1e3,1), round(d['roofline']['avg_launch_ms']*1e3,1))" \
      gpurun_out/ab/${VAR}_${v}_$r.json "$VAR=$v"
  done
done
