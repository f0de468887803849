#!/bin/bash
# Diagnostic library variants (same sources, different -D switches) into build/.
# usage: tools/build_variants.sh NAME "-DFLAG=.. -DFLAG2=.." [NAME2 "FLAGS2" ...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/mfgp_coverage_amd/csrc
mkdir -p $R/build
while [ $# -ge 2 ]; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC $2 -o $R/build/libmfgp_$1.so \
    $C/mfgp_kernels.hip $C/mfgp_cells.hip $C/mfgp_nlml.hip $C/mfgp_capi.hip &
  shift 2
done
wait
ls -la $R/build
