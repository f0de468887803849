#!/bin/bash
# g3 timeline (stamps build) with and without the K loop's B loads
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
MFGP_LAT_G3=1 timeout -k 10 200 python -u tools/trace_g3.py tools/diaglib/libmfgp_stamps.so | tail -6 || exit 1
echo "== no B loads"
MFGP_LAT_G3=1 timeout -k 10 200 python -u tools/trace_g3.py tools/diaglib/libmfgp_stamps_nob.so | tail -6
