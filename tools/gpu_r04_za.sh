#!/bin/bash
# headline: member-list Z units (MFGP_LAT_ZCSR=1) vs the bucketing ones (default there), alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2 3; do
  for z in 0 1; do
    MFGP_LAT_ZCSR=$z timeout -k 10 300 python bench.py --no-full --no-cpu-baseline --sim-iterations 0 > gpurun_out/r04za_h${z}_$rep.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/r04za_h${z}_$rep.json')); print('zcsr=$z rep $rep', round(d['value']), round(1e3*d['ms_per_step'],2), round(1e3*d['roofline']['avg_launch_ms'],2))"
  done
done
