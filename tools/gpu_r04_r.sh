#!/bin/bash
# w units balanced by priority-by-progress (wprio) or by skewed shares (wskew75): per-unit timelines, then the headline A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for v in wprio wskew75; do
  timeout -k 10 200 python -u tools/trace_lat.py tools/diaglib/libmfgp_stamps_$v.so > gpurun_out/r04r_trace_$v.txt 2>&1 || exit 1
  echo "== $v"; grep "w units published" gpurun_out/r04r_trace_$v.txt
  grep -A65 "index, start" gpurun_out/r04r_trace_$v.txt | awk 'NR>1{s+=$3; if($4>m)m=$4; if(NR<=33){a+=$3}else{b+=$3}} END{print "mean dur", s/(NR-1), "first half", a/32, "second half", b/32, "max end", m}'
done
bash tools/ab_variants.sh wprio wskew75
