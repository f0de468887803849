#!/bin/bash
# round-4: concurrency A/B of the headline step (1, 2, 4 sub-batch streams)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for ns in 1 2 4; do
  timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --no-full --no-cpu-baseline --sim-iterations 0 --streams $ns \
    > gpurun_out/r04b_streams$ns.json 2> gpurun_out/r04b_streams$ns.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/r04b_streams$ns.json'));print($ns, d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline'].get('step_aggregate_frac'))"
done
